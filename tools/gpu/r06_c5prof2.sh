# round 6: the data-parallel C5 step under latency injection (W = 4): timed-window length vs
# step time, and a kernel trace of the steady state (whole-epoch warm-up)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/r06c5p2}
mkdir -p "$OUT"
for S in 12 30; do
  timeout -k 10 400 env RSX_COMM_SIM=4 python bench.py --workload c5 --steps $S --warmup 6 --no-cpu-baseline \
    > "$OUT/sim4_s$S.json" 2> "$OUT/sim4_s$S.err" || { tail -20 "$OUT/sim4_s$S.err"; exit 1; }
  grep "bench\]" "$OUT/sim4_s$S.err"
done
timeout -k 10 500 env RSX_COMM_SIM=4 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/tr" -o t -- \
  python bench.py --workload c5 --steps 30 --warmup 6 --no-cpu-baseline > "$OUT/tr.json" 2> "$OUT/tr.err" || { tail -20 "$OUT/tr.err"; exit 1; }
grep "bench\]" "$OUT/tr.err"
echo done
