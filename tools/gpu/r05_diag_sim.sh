# round 5: which latency-injected Comm pattern breaks a graph capture (the C5 sim leg
# segfaulted in capture_end)?  Patterns one process each, stopping at the first failure
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONFAULTHANDLER=1 RSX_COMM_SIM=4
OUT=${OUT:-gpurun_out/r05diag}
mkdir -p $OUT
for p in ${PATTERNS:-ar ag side grad all}; do
  timeout -k 10 120 python -X faulthandler tools/gpu/diag_smore_sim.py $p > $OUT/diag_$p.txt 2>&1
  rc=$?; echo "$p rc=$rc"; tail -3 $OUT/diag_$p.txt
  [ $rc -eq 0 ] || exit $rc
done
# every pattern captured: the step itself, eager (no graph) then captured
RSX_BENCH_GRAPH=0 timeout -k 10 300 python -X faulthandler bench.py --workload c5 --steps 4 --warmup 2 \
  --no-cpu-baseline > $OUT/c5_eager.json 2> $OUT/c5_eager.err; rc=$?; echo "c5 eager rc=$rc"; tail -5 $OUT/c5_eager.err
echo done
