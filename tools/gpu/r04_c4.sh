# round 4: C4 strong scaling measured on one GPU under latency injection (RSX_COMM_SIM,
# csrc/dist.hip rsx_comm_init_sim): rank 0's share of a W-rank job (8/W user chunks, batch
# 2048/W), every collective a comm-stream kernel holding the modelled time, 32 workgroups
# and the collective's HBM bytes at W ranks; the same share with no exchange (compute
# only); the head-piece A/B at W = 8; then the full 10M-user graph on one GPU (the N = 1
# anchor) with its CPU baseline.  PART=1: W = 8, 4, 2; PART=2: the N = 1 anchor.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r04c4}
mkdir -p $OUT
A="--workload c4 --steps ${STEPS:-8} --warmup 2 --no-cpu-baseline --eval-users 4096"
summ() {
  python -c "
import json, sys
d = json.load(open('$OUT/$1.json'))
li = d.get('latency_injection') or {}
print('$1', 'ms/step', round(d['ms_per_step'], 3), 'value', round(d['value'], 1), li.get('per_collective_ms', ''), li.get('measured_allreduce_item_block_ms', ''))"
}
run() {  # name, timeout, env..., -- args
  local name=$1 to=$2; shift 2
  timeout -k 10 $to env "$@" python bench.py $A $EXTRA > $OUT/$name.json 2> $OUT/$name.err || { tail -20 $OUT/$name.err; return 1; }
  summ $name
}
if [ "${PART:-1}" = 1 ]; then
EXTRA="" run sim_w8 500 RSX_COMM_SIM=8 || exit 1
EXTRA="" run sim_w8_head4 500 RSX_COMM_SIM=8 RSX_SHARDED_HEAD=4 || exit 1
EXTRA="--c4-chunks 1 --batch 256" run compute_w8 500 RSX_X=0 || exit 1
EXTRA="" run sim_w4 600 RSX_COMM_SIM=4 || exit 1
EXTRA="--c4-chunks 2 --batch 512" run compute_w4 600 RSX_X=0 || exit 1
EXTRA="" run sim_w2 800 RSX_COMM_SIM=2 || exit 1
EXTRA="--c4-chunks 4 --batch 1024" run compute_w2 800 RSX_X=0 || exit 1
fi
if [ "${PART:-1}" = 2 ]; then
# the N = 1 anchor: the whole 10M-user graph on one GPU, with its CPU baseline
timeout -k 10 1000 python bench.py --workload c4 --steps 6 --warmup 2 --eval-users 4096 --cpu-budget 20 > $OUT/full_n1.json 2> $OUT/full_n1.err || { tail -20 $OUT/full_n1.err; exit 1; }
summ full_n1
fi
echo done
