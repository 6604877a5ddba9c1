# round 4: C4 strong scaling under latency injection (RSX_COMM_SIM, csrc/dist.hip
# rsx_comm_init_sim): rank 0's share of a W-rank job on ONE GPU (8/W user chunks, batch
# 2048/W) with every collective a comm-stream kernel of the modelled time / CUs / HBM
# bytes at W ranks.  Plus the same shares without exchanges (pure compute).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/c4sim}
mkdir -p $OUT
A="--workload c4 --steps ${STEPS:-8} --warmup 2 --no-cpu-baseline --eval-users 4096"
for W in ${WS:-8 4 2}; do
  C=$((8 / W))
  RSX_COMM_SIM=$W timeout -k 10 500 python bench.py $A > $OUT/sim_w$W.json 2> $OUT/sim_w$W.err || { tail -20 $OUT/sim_w$W.err; exit 1; }
  timeout -k 10 500 python bench.py $A --c4-chunks $C --batch $((2048 / W)) > $OUT/compute_w$W.json 2> $OUT/compute_w$W.err || { tail -20 $OUT/compute_w$W.err; exit 1; }
  python -c "
import json
s=json.load(open('$OUT/sim_w$W.json')); c=json.load(open('$OUT/compute_w$W.json'))
print('W=$W', 'sim ms/step', round(s['ms_per_step'],2), 'compute-only ms/step', round(c['ms_per_step'],2), s['latency_injection']['per_collective_ms'])"
done
