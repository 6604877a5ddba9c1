# round 4, batch D: the sharded-step GPU tests (neighbour-row exchange of the last forward
# layer, owner Adam on the comm stream), then C4 under latency injection: W = 8 with / without
# the neighbour exchange and graph-replayed / eager, W = 4 and 2, and a W = 8 step trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r04d}
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
run sim_w8_eager RSX_COMM_SIM=8 RSX_SHARDED_GRAPH=0 || exit 1
run sim_w8_nonbr RSX_COMM_SIM=8 RSX_SHARDED_NBR=0 || exit 1
run sim_w8_adam_compute RSX_COMM_SIM=8 RSX_SHARDED_COMM_ADAM=0 || exit 1
run sim_w8_head1 RSX_COMM_SIM=8 RSX_SHARDED_HEAD=1 || exit 1
run sim_w4 RSX_COMM_SIM=4 || exit 1
run sim_w2 RSX_COMM_SIM=2 || exit 1
W=8 OUT=$OUT/trace_w8 bash tools/gpu/c4_simtrace.sh
echo done
