# round 6: what costs the data-parallel C5 step its extra time under latency injection
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/r06c5d}
mkdir -p "$OUT"
run() {  # name, env...
  local name=$1; shift
  timeout -k 10 400 env "$@" python bench.py --workload c5 --steps 12 --warmup 6 --no-cpu-baseline \
    > "$OUT/$name.json" 2> "$OUT/$name.err" || { tail -20 "$OUT/$name.err"; return 1; }
  echo "$name $(grep 'bench\]' "$OUT/$name.err")"
}
run sim4 RSX_COMM_SIM=4 || exit 1
run sim4_free RSX_COMM_SIM=4:1000000:0:1 || exit 1
run sim4_nostreams RSX_COMM_SIM=4 RSX_SMORE_STREAMS=0 || exit 1
run sim4_eager RSX_COMM_SIM=4 RSX_BENCH_GRAPH=0 || exit 1
run n1_nostreams RSX_SMORE_STREAMS=0 || exit 1
run dp1_eager RSX_BENCH_SHARDED=1 || exit 1
echo done
