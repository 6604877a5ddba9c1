# full GPU suite (one process), smoke, then the default bench line and every
# single-GPU leg without the CPU baseline (ms/step per leg on stdout)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/verify}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
for w in ${LEGS:-c2 baby c1 c3 c5}; do
  timeout -k 10 400 python bench.py --workload $w --no-cpu-baseline > $OUT/$w.json 2> $OUT/$w.err || { tail -20 $OUT/$w.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$w.json')); print('$w', round(d['ms_per_step'],4), 'ms/step', round(d['value']))"
done
