# round 6: kernel traces of the C5 step: one GPU, the data-parallel model on one real rank
# (exchange work, no collective) and under latency injection (W = 4)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/r06c5p}
mkdir -p "$OUT"
A="--workload c5 --steps 12 --warmup 6 --no-cpu-baseline"
prof() {  # name, env...
  local name=$1; shift
  timeout -k 10 400 env "$@" rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$name" -o t -- \
    python bench.py $A > "$OUT/$name.json" 2> "$OUT/$name.err" || { tail -20 "$OUT/$name.err"; return 1; }
  grep "bench\]" "$OUT/$name.err"
}
prof n1 RSX_X=0 || exit 1
prof dp1 RSX_BENCH_SHARDED=1 || exit 1
prof dpsim4 RSX_COMM_SIM=4 || exit 1
echo done
