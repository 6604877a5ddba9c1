# A/B on one box: each leg with the default build settings and with RSX_SPMM_MAXB=$B
# (interleaved, twice), ms/step per run on stdout
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/ab}
B=${B:-2048}
mkdir -p $OUT
for w in ${LEGS:-baby c1 c2}; do
  for rep in 1 2; do
    for m in default $B; do
      if [ $m = default ]; then unset RSX_SPMM_MAXB; else export RSX_SPMM_MAXB=$m; fi
      timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > $OUT/$w.$m.$rep.json 2> $OUT/$w.$m.$rep.err || { tail -20 $OUT/$w.$m.$rep.err; exit 1; }
      python -c "import json; d=json.load(open('$OUT/$w.$m.$rep.json')); print('$w', '$m', $rep, round(d['ms_per_step']*1e3,2), 'us/step')"
    done
  done
done
