# round 4: the fused projection backward (wgrad_partial DX) with its LDS operands read
# ahead of the MFMAs: the linear / SMORE tests, then C5 / C3 timings (roofline_kernels
# carries rsx_linear_bwd's live average) beside the base variant
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r04lin}
mkdir -p $OUT; rm -f $OUT/t.txt
VB=recommendar-systems_amd/rsx/lib/variants/base/librsx.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_smore.py tests/test_gpu_smore_fuse.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in base new; do
    unset RSX_LIB; [ $v = base ] && export RSX_LIB=$VB
    for w in c5 c3; do
      timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --steps 30 --warmup 6 > $OUT/${w}_${v}_$rep.json 2> $OUT/${w}_${v}_$rep.err || exit 1
      python -c "import json;d=json.load(open('$OUT/${w}_${v}_$rep.json'));print('$w $v $rep', round(d['ms_per_step'],4), [(k['kernel'][:14], round(k.get('avg_launch_ms',0)*1e3,1)) for k in d.get('roofline_kernels',[])][:1])" >> $OUT/t.txt
    done
  done
done
cat $OUT/t.txt
