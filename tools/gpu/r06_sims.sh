# round 6: latency-injected legs (RSX_COMM_SIM=W on one GPU: rank 0 of a modelled W-rank job,
# every collective a comm-stream stand-in of its modelled time, 32 CUs and HBM bytes) beside
# their N = 1 lines.  PART: c5 (data-parallel SMORE, both link models), c2row (the row-sharded
# C2 weak leg), c4d64 (LightGCN d=64 on the 10M-user graph, strong), dpref (one-GPU comparators
# of the DP leg at B = W x 2048)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONFAULTHANDLER=1
OUT=${OUT:-gpurun_out/r06sims}
mkdir -p "$OUT"
summ() {
  python -c "
import json
d = json.load(open('$OUT/$1.json'))
li = d.get('latency_injection') or {}
print('$1', 'ms/step', round(d['ms_per_step'], 4), 'value', round(d['value'], 1), 'job', li.get('modelled_job'))"
}
run() {  # name, timeout, env...  (bench args in ARGS)
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" env "$@" python bench.py $ARGS > "$OUT/$name.json" 2> "$OUT/$name.err" || { tail -20 "$OUT/$name.err"; return 1; }
  summ "$name"
}
bw6() { python -c "print(min($1 - 1, 7) * 76.5 * 0.6)"; }
for part in ${PART:-c5}; do
case $part in
c5)
  ARGS="--workload c5 --steps 30 --warmup 6 --no-cpu-baseline"
  run c5_n1 600 RSX_X=0 || exit 1
  for W in 2 4 8; do run c5_dp_sim_w$W 600 RSX_COMM_SIM=$W || exit 1; done
  for W in 2 4 8; do run c5_dp_sim06_w$W 600 RSX_COMM_SIM=$W:$(bw6 $W) || exit 1; done
  ;;
c5us)
  ARGS="--workload c5 --steps 30 --warmup 6 --no-cpu-baseline"
  for W in 2 4; do run c5_us_sim_w$W 600 RSX_SMORE_SCHEME=usershard RSX_COMM_SIM=$W || exit 1; done
  ;;
c3)
  ARGS="--workload c3 --steps 30 --warmup 6 --no-cpu-baseline"
  run c3_n1 600 RSX_X=0 || exit 1
  for W in 2 8; do run c3_dp_sim_w$W 600 RSX_COMM_SIM=$W || exit 1; done
  ;;
c2row)
  ARGS="--steps 300 --warmup 30 --no-cpu-baseline"
  for W in 2 4 8; do run c2row_sim_w$W 400 RSX_COMM_SIM=$W || exit 1; done
  for W in 2 8; do run c2row_sim06_w$W 400 RSX_COMM_SIM=$W:$(bw6 $W) || exit 1; done
  ;;
dpref)
  ARGS="--steps 300 --warmup 30 --no-cpu-baseline"
  for B in 4096 8192 16384; do ARGS="--steps 300 --warmup 30 --no-cpu-baseline --batch $B"; run c2_b$B 400 RSX_X=0 || exit 1; done
  ;;
c4d64)
  ARGS="--workload c4 --dim 64 --steps 10 --warmup 3 --eval-users 4096"
  run c4d64_n1 900 RSX_X=0 || exit 1
  ARGS="--workload c4 --dim 64 --steps 10 --warmup 3 --eval-users 4096 --no-cpu-baseline"
  for W in 2 4 8; do run c4d64_sim_w$W 900 RSX_COMM_SIM=$W || exit 1; done
  for W in 2 8; do run c4d64_sim06_w$W 900 RSX_COMM_SIM=$W:$(bw6 $W) || exit 1; done
  ;;
esac
done
echo done
