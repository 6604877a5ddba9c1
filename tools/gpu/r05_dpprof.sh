# round 5: kernel traces of the triplets-only DP step (and the C5 step's launch sequence) (one real RCCL rank; rank 0 of a
# latency-injected 8-rank job) beside the single-GPU C2 engine, for the per-launch breakdown
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05dpprof}
mkdir -p $OUT
prof() {  # name, env..., -- bench args in ARGS
  local name=$1; shift
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$name -o $name -- python3 bench.py $ARGS \
    > $OUT/$name.json 2> $OUT/$name.err || { tail -20 $OUT/$name.err; return 1; }
  python3 tools/kstats.py $(find $OUT/$name -name "*kernel_stats.csv" | head -1) 2>/dev/null | head -30 || true
}
ARGS="--steps 200 --warmup 20 --no-cpu-baseline"
prof c2 RSX_X=0 || exit 1
ARGS="--dp --steps 200 --warmup 20 --no-cpu-baseline"
prof dp1 RSX_X=0 || exit 1
prof dp_sim8 RSX_COMM_SIM=8 || exit 1
# the C5 step's launch sequence (every dispatch, 3 timed steps): where its fills and small
# kernels sit
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/c5seq -o c5seq -- python3 bench.py --workload c5 \
  --steps 3 --warmup 2 --no-cpu-baseline > $OUT/c5seq.json 2> $OUT/c5seq.err || { tail -20 $OUT/c5seq.err; exit 1; }
echo done
