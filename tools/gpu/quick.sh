# quick iteration: selected GPU tests (pytest -k "$K"), then the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/quick}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "${K:-.}" > $OUT/pytest.log 2>&1
rc=$?; tail -15 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$BENCH" ]; then
  timeout -k 10 400 python bench.py $BENCH > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
  cat $OUT/bench.json
fi
