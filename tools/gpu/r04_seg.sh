# round 4: pref_segsum with its row scans issuing several chunk loads at a time (first run:
# against the HEAD variant, gpurun_out/r04seg), then with the row ids in LDS (VARIANT=env:
# RSX_SEGSUM_GLOBAL=1 as the 'head' leg instead of a build): the SMORE tests, C5 / C3, C5 kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r04seg}
mkdir -p $OUT; rm -f $OUT/t.txt
VH=recommendar-systems_amd/rsx/lib/variants/head/librsx.so
timeout -k 10 500 python -u -m pytest tests/test_gpu_smore.py tests/test_gpu_smore_fuse.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in head new; do
    unset RSX_LIB RSX_SEGSUM_GLOBAL
    if [ $v = head ]; then if [ "$VARIANT" = env ]; then export RSX_SEGSUM_GLOBAL=1; else export RSX_LIB=$VH; fi; fi
    for w in c5 c3; do
      timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --steps 30 --warmup 6 > $OUT/${w}_${v}_$rep.json 2> $OUT/${w}_${v}_$rep.err || exit 1
      python -c "import json;d=json.load(open('$OUT/${w}_${v}_$rep.json'));print('$w $v $rep', round(d['ms_per_step'],4))" >> $OUT/t.txt
    done
  done
done
for v in head new; do
  unset RSX_LIB RSX_SEGSUM_GLOBAL
  if [ $v = head ]; then if [ "$VARIANT" = env ]; then export RSX_SEGSUM_GLOBAL=1; else export RSX_LIB=$VH; fi; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_$v -o c5 -- python bench.py --workload c5 --no-cpu-baseline --steps 20 --warmup 6 > $OUT/c5prof_$v.json 2> $OUT/c5prof_$v.err || exit 1
done
find $OUT -name '*kernel_trace.csv' -delete
cat $OUT/t.txt
grep -h "pref_segsum\|pref_bwd_rows" $OUT/stats_*/c5_kernel_stats.csv | cut -d, -f1-4
