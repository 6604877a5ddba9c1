# round 5, fourth GPU batch: the DP step with the slot pack on the comm branch, whole-chunk
# gathers, wave-aggregated run reservation, fence-free sc1 loss hand-offs (dp_bpr_coef and
# the single-GPU bpr_fused); the spectral backward in two wave halves.  Tests, then the
# C2 / DP legs, a DP kernel trace, and the C5 / C3 lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONFAULTHANDLER=1
OUT=${OUT:-gpurun_out/r05b4}
mkdir -p $OUT
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_smore.py tests/test_gpu_kernels.py -m gpu -v \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" $OUT/pytest.log | tail -15; ok $rc || exit $rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/gpu/micro_item.py > $OUT/micro_item.txt 2>&1 || exit 1
cat $OUT/micro_item.txt
OUT=$OUT PART=dp bash tools/gpu/r05_sims.sh || exit 1
RSX_COMM_SIM=8 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/dp_sim8_trace -o t -- \
  python3 bench.py --dp --steps 60 --warmup 20 --no-cpu-baseline > $OUT/dp_sim8_trace.json 2> $OUT/dp_sim8_trace.err \
  || { tail -20 $OUT/dp_sim8_trace.err; exit 1; }
for w in c5 c3; do
  timeout -k 10 600 python bench.py --workload $w --steps 30 --warmup 6 --no-cpu-baseline > $OUT/$w.json 2> $OUT/$w.err \
    || { tail -20 $OUT/$w.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$w.json')); print('$w', round(d['ms_per_step'], 4), 'ms/step')"
done
