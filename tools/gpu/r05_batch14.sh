# round 5, fourteenth GPU batch: the DP loss passes' middle lane-group form at W = 4 (2
# triplets / 8 run places a group for 8192 <= W B < 16384); the projection backward's dW
# and db partials reduced in one launch.  DP tests (three forms), the DP legs; the SMORE
# / linear GPU tests, the projection micro-benchmark, the C5 / C3 lines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONFAULTHANDLER=1
OUT=${OUT:-gpurun_out/r05b14}
mkdir -p $OUT
timeout -k 10 800 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_smore.py tests/test_gpu_smore_fuse.py \
  tests/test_gpu_kernels.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" $OUT/pytest.log | tail -12; [ $rc -eq 0 ] || exit $rc
OUT=$OUT PART=dp bash tools/gpu/r05_sims.sh || exit 1
timeout -k 10 120 python tools/gpu/micro_gemm.py > $OUT/micro_gemm.json 2> $OUT/micro_gemm.err || exit 1
cat $OUT/micro_gemm.json
for w in c5 c3; do
  timeout -k 10 300 python bench.py --workload $w --steps 30 --warmup 6 --no-cpu-baseline > $OUT/$w.json 2> $OUT/$w.err || exit 1
  python -c "import json;d=json.load(open('$OUT/$w.json'));print('$w', d['ms_per_step'])"
done
echo done
