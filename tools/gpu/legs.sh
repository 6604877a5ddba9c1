# every bench leg with its rocprofv3 kernel-stats summary (round 2): LEGS="c2 baby c1 c3 c5" OUT=gpurun_out/legs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/legs}
mkdir -p $OUT
for w in ${LEGS:-c2 baby c1 c3 c5}; do
  echo "== $w $(date +%T)"
  timeout -k 10 ${TLEG:-400} python bench.py --workload $w ${ARGS:-} > $OUT/$w.json 2> $OUT/$w.err || { echo "bench $w failed rc=$?"; tail -20 $OUT/$w.err; exit 1; }
  cat $OUT/$w.json
  if [ -z "${NOPROF:-}" ]; then
    timeout -k 10 ${TLEG:-400} rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$w -o $w -- python3 bench.py --workload $w --no-cpu-baseline ${PARGS:---steps 50 --warmup 10} > $OUT/prof_$w.json 2> $OUT/prof_$w.err || { echo "prof $w failed rc=$?"; tail -20 $OUT/prof_$w.err; exit 1; }
  fi
  # keep the summaries only (traces are large; gpurun_out is capped at 64 MiB)
  find $OUT -type f ! -name '*kernel_stats.csv' ! -name '*.json' ! -name '*.err' -delete
done
echo done
