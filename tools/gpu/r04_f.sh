# round 4, batch F: sharded-step GPU tests with the deferred parameter all-gather, then C4
# at the modelled W = 8 / 4 / 2 jobs (defaults) and W = 8 without the deferral
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r04f}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_sharded_trainer.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
A="--workload c4 --steps 8 --warmup 2 --no-cpu-baseline --eval-users 4096"
run() {  # name, env...
  local name=$1; shift
  timeout -k 10 500 env "$@" python bench.py $A > $OUT/$name.json 2> $OUT/$name.err || { tail -20 $OUT/$name.err; return 1; }
  python -c "
import json
d = json.load(open('$OUT/$name.json'))
li = d.get('latency_injection') or {}
print('$name', 'ms/step', round(d['ms_per_step'], 3), li.get('measured_allreduce_item_block_ms', ''))"
}
run sim_w8 RSX_COMM_SIM=8 || exit 1
run sim_w8_nodefer RSX_COMM_SIM=8 RSX_SHARDED_DEFER_AG=0 || exit 1
run sim_w4 RSX_COMM_SIM=4 || exit 1
run sim_w2 RSX_COMM_SIM=2 || exit 1
W=8 OUT=$OUT/trace_w8 bash tools/gpu/c4_simtrace.sh
echo done
