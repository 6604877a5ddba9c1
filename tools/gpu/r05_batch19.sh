# round 5, nineteenth GPU batch: the bench's data-parallel leg at 2 and 4 ranks on the one
# GPU (gloo host-hook collectives: RCCL refuses two ranks on one GPU) -- the N-rank launch,
# the eager DP step, and the new cross-rank bit-identity check of the replicas
# (dp_replicas_bit_identical in the line); a rehearsal of the code path, not a measurement
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONFAULTHANDLER=1
OUT=${OUT:-gpurun_out/r05b19}
mkdir -p $OUT
for n in 2 4; do
  RSX_BENCH_SAME_DEVICE=1 RSX_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus $n --steps 20 --warmup 5 \
    --no-cpu-baseline > $OUT/dp_gloo_n$n.json 2> $OUT/dp_gloo_n$n.err || { tail -20 $OUT/dp_gloo_n$n.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/dp_gloo_n$n.json'));print('n=$n', d['config']['parallelism'], 'replicas identical:', d.get('dp_replicas_bit_identical'), 'rccl_world', d.get('rccl_world_size'))"
done
echo done
