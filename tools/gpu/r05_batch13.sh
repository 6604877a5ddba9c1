# round 5, thirteenth GPU batch: the DP loss passes' lane-group sizes at W = 4 / 8
# (latency-injected; RSX_DP_TPG triplets, RSX_DP_CH run places a group) against the default
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONFAULTHANDLER=1
OUT=${OUT:-gpurun_out/r05b13}
mkdir -p $OUT
ARGS="--dp --steps 300 --warmup 30 --no-cpu-baseline"
run() {  # name, env...
  local name=$1; shift
  timeout -k 10 200 env "$@" python bench.py $ARGS > $OUT/$name.json 2> $OUT/$name.err || { tail -20 $OUT/$name.err; return 1; }
  python -c "import json;d=json.load(open('$OUT/$name.json'));print('$name', round(d['ms_per_step'],4))"
}
for W in 8 4; do
  run w${W}_default RSX_COMM_SIM=$W || exit 1
  run w${W}_t2c8 RSX_COMM_SIM=$W RSX_DP_TPG=2 RSX_DP_CH=8 || exit 1
  run w${W}_t4c8 RSX_COMM_SIM=$W RSX_DP_TPG=4 RSX_DP_CH=8 || exit 1
  run w${W}_t1c4 RSX_COMM_SIM=$W RSX_DP_TPG=1 RSX_DP_CH=4 || exit 1
  run w${W}_t2c16 RSX_COMM_SIM=$W RSX_DP_TPG=2 RSX_DP_CH=16 || exit 1
done
run w2_default RSX_COMM_SIM=2 || exit 1
run w2_t2c8 RSX_COMM_SIM=2 RSX_DP_TPG=2 RSX_DP_CH=8 || exit 1
run n1_t2c8 RSX_X=0 RSX_DP_TPG=2 RSX_DP_CH=8 || exit 1
echo done
