# round 5: kernel traces (every dispatch, CSV) of the DP step after the gradient-pass and
# bucketing changes: one real RCCL rank, and rank 0 of a latency-injected 8-rank job
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05dpprof2}
mkdir -p $OUT
prof() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$name -o $name -- \
    python3 bench.py --dp --steps 100 --warmup 20 --no-cpu-baseline > $OUT/$name.json 2> $OUT/$name.err \
    || { tail -20 $OUT/$name.err; return 1; }
}
prof dp1 RSX_X=0 || exit 1
prof dp_sim8 RSX_COMM_SIM=8 || exit 1
echo done
