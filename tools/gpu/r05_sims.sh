# round 5: the data-parallel C2 leg and the embed-sharded C5 leg under latency injection
# (RSX_COMM_SIM=W on one GPU: rank 0 of a modelled W-rank job, every collective a comm-stream
# stand-in holding its modelled time, 32 CUs and HBM bytes), beside their N = 1 lines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONFAULTHANDLER=1
OUT=${OUT:-gpurun_out/r05sims}
mkdir -p $OUT
summ() {
  python -c "
import json
d = json.load(open('$OUT/$1.json'))
li = d.get('latency_injection') or {}
print('$1', 'ms/step', round(d['ms_per_step'], 4), 'value', round(d['value'], 1), 'job', li.get('modelled_job'), li.get('per_collective_ms', ''))"
}
run() {  # name, timeout, env..., -- (bench args in ARGS)
  local name=$1 to=$2; shift 2
  timeout -k 10 $to env "$@" python bench.py $ARGS > $OUT/$name.json 2> $OUT/$name.err || { tail -20 $OUT/$name.err; return 1; }
  summ $name
}
if [ "${PART:-dp}" = dp ]; then
ARGS="--steps 300 --warmup 30 --no-cpu-baseline"
run c2_n1 300 RSX_X=0 || exit 1
ARGS="--dp --steps 300 --warmup 30 --no-cpu-baseline"
run dp_n1 300 RSX_X=0 || exit 1
for W in 2 4 8; do run dp_sim_w$W 300 RSX_COMM_SIM=$W || exit 1; done
fi
if [ "${PART:-dp}" = dpeager ]; then  # the DP step issued eagerly (no graph replay)
ARGS="--dp --steps 300 --warmup 30 --no-cpu-baseline"
run dp_eager_n1 300 RSX_DP_GRAPH=0 || exit 1
for W in 2 8; do run dp_eager_sim_w$W 300 RSX_DP_GRAPH=0 RSX_COMM_SIM=$W || exit 1; done
fi
if [ "${PART:-dp}" = solo ]; then  # one real rank: the comm branch in line vs forked
ARGS="--dp --steps 300 --warmup 30 --no-cpu-baseline"
for i in 1 2; do
  run dp_solo_n1_$i 300 RSX_DP_SOLO=1 || exit 1
  run dp_forked_n1_$i 300 RSX_DP_SOLO=0 || exit 1
done
fi
if [ "${PART:-dp}" = places ]; then  # W > 1: the run places taken in the loss pass vs dp_scatter
ARGS="--dp --steps 300 --warmup 30 --no-cpu-baseline"
for W in 2 4 8; do
  run dp_sim_w${W}_inloss 300 RSX_COMM_SIM=$W RSX_DP_PLACES_IN_LOSS=1 || exit 1
  run dp_sim_w${W}_scatter 300 RSX_COMM_SIM=$W RSX_DP_PLACES_IN_LOSS=0 || exit 1
  run dp_sim_w${W}_inloss2 300 RSX_COMM_SIM=$W RSX_DP_PLACES_IN_LOSS=1 || exit 1
  run dp_sim_w${W}_scatter2 300 RSX_COMM_SIM=$W RSX_DP_PLACES_IN_LOSS=0 || exit 1
done
fi
if [ "${PART:-dp}" = c5 ]; then
ARGS="--workload c5 --steps 30 --warmup 6 --no-cpu-baseline"
run c5_n1 600 RSX_X=0 || exit 1
for W in 4 2 8; do run c5_sim_w$W 600 RSX_COMM_SIM=$W || exit 1; done
fi
echo done
