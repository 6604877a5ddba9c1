# round 5, seventh GPU batch: the DP loss pass with four triplets per lane group (row gathers
# batched, the last block's partial loads in one round) and the exact power-of-two
# reciprocal in the gradient pass; the projection backward with conflict-free LDS layouts.
# DP + linear tests, the projection micro-benchmark, the DP legs (graph replay and eager),
# a DP kernel trace at a latency-injected W = 8, the C5 line, and the C5 step's collectives
# at a latency-injected W = 2 (kernel stats)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONFAULTHANDLER=1
OUT=${OUT:-gpurun_out/r05b7}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_smore.py -m gpu -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider -k "dp or linear or wgrad or proj" > $OUT/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" $OUT/pytest.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/gpu/micro_gemm.py > $OUT/micro_gemm.json 2> $OUT/micro_gemm.err || exit 1
cat $OUT/micro_gemm.json
OUT=$OUT PART=dp bash tools/gpu/r05_sims.sh || exit 1
OUT=$OUT PART=dpeager bash tools/gpu/r05_sims.sh || exit 1
RSX_COMM_SIM=8 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace8 -o t -- \
  python3 bench.py --dp --steps 60 --warmup 20 --no-cpu-baseline > $OUT/trace8.json 2> $OUT/trace8.err \
  || { tail -20 $OUT/trace8.err; exit 1; }
timeout -k 10 300 python bench.py --workload c5 --steps 30 --warmup 6 --no-cpu-baseline > $OUT/c5.json 2> $OUT/c5.err || exit 1
python -c "import json;d=json.load(open('$OUT/c5.json'));print('c5', d['ms_per_step'])"
RSX_COMM_SIM=2 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c5sim2 -o t -- \
  python3 bench.py --workload c5 --steps 6 --warmup 3 --no-cpu-baseline > $OUT/c5sim2.json 2> $OUT/c5sim2.err \
  || { tail -20 $OUT/c5sim2.err; exit 1; }
echo done
