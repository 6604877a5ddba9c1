# rocprofv3 kernel stats of one bench leg: LEG=c3 OUT=gpurun_out/pl
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pl}
mkdir -p $OUT
for w in ${LEGS:-c3}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$w -o $w -- python3 bench.py --workload $w --no-cpu-baseline ${PARGS:---steps 30 --warmup 6} > $OUT/$w.json 2> $OUT/$w.err || { tail -20 $OUT/$w.err; exit 1; }
  cat $OUT/$w.json
  find $OUT -name '*kernel_trace.csv' -delete
done
