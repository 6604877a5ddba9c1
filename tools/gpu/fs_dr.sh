# fs_screen per-phase times: drain widths (variants dr1 / main = 2 / dr4), then exactness tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/fsdr}
mkdir -p $OUT
for v in dr1 main dr4; do
  if [ $v = main ]; then unset RSX_LIB; else export RSX_LIB=recommendar-systems_amd/rsx/lib/variants/$v/librsx.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v -o run -- python tools/gpu/fsbal.py 35598 > $OUT/$v.log 2>&1 || exit 1
  echo "== $v"; grep nb= $OUT/$v.log
  python tools/kstats.py $(find $OUT/$v -name '*kernel_stats.csv') 3
  find $OUT/$v -name '*kernel_trace.csv' -delete
done
unset RSX_LIB
timeout -k 10 300 python -u -m pytest tests/test_gpu_realshape.py tests/test_gpu_kernels.py -m gpu -x -q -k "fullsort or screen or topk" --timeout 200 --timeout-method thread > $OUT/pytest.txt 2>&1
tail -n 2 $OUT/pytest.txt
