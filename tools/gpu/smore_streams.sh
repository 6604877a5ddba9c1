# SMORE: GPU tests, then the C3 / C5 legs with the UI backbone on a side stream and
# without (RSX_SMORE_STREAMS=0), with the dominant-kernel rooflines of each line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/sst}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_smore.py tests/test_gpu_smore_dist.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for w in c5 c3; do
  for st in 1 0; do
    RSX_SMORE_STREAMS=$st timeout -k 10 300 python bench.py --workload $w --steps 60 --warmup 10 --no-cpu-baseline > $OUT/${w}_s$st.json 2> $OUT/${w}_s$st.err || { tail -20 $OUT/${w}_s$st.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/${w}_s$st.json')); print('$w streams=$st', round(d['value']), round(d['ms_per_step'], 3)); [print('   ', r['kernel'][:60], round(r['avg_launch_ms']*1e3,1), 'us', round(r['frac'],3)) for r in d['roofline_kernels']]"
  done
done
