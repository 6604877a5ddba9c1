# round 5: the C4 strong-scaling sims (tools/gpu/r04_c4.sh) at two more link models:
# MODEL=eff06 — ring efficiency 0.6 instead of 0.8 (bus bandwidth min(W-1,7) x 76.5 GB/s x 0.6:
# 45.9 / 137.7 / 321.3 GB/s at W = 2 / 4 / 8); MODEL=lat50 — 50 us per collective instead of 30
# (0.8 efficiency).  N = 1 anchor: profiles/r04/c4/final/full_n1.json (144.7 ms/step).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05c4}
mkdir -p $OUT
A="--workload c4 --steps ${STEPS:-8} --warmup 2 --no-cpu-baseline --eval-users 4096"
summ() {
  python -c "
import json
d = json.load(open('$OUT/$1.json'))
li = d.get('latency_injection') or {}
print('$1', 'ms/step', round(d['ms_per_step'], 3), li.get('busbw_gbs'), li.get('latency_us'), li.get('per_collective_ms', ''), li.get('measured_allreduce_item_block_ms', ''))"
}
run() {  # name, timeout, env...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to env "$@" python bench.py $A > $OUT/$name.json 2> $OUT/$name.err || { tail -20 $OUT/$name.err; return 1; }
  summ $name
}
for m in ${MODELS:-eff06 lat50}; do
  for W in 8 4 2; do
    L=$(( W - 1 < 7 ? W - 1 : 7 ))
    if [ $m = eff06 ]; then bw=$(python -c "print($L * 76.5 * 0.6)"); lat=30; else bw=$(python -c "print($L * 76.5 * 0.8)"); lat=50; fi
    run sim_${m}_w$W 900 RSX_COMM_SIM=$W:$bw:$lat || exit 1
  done
done
echo done
