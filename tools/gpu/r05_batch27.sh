# round 5, twenty-seventh GPU batch: tagged-row SpMM launches issuing U work items'
# descriptor + tag loads together (RSX_SPMM_TAG_BATCH = 4, the default build; 1 = the
# one-at-a-time walk, 8) -- the GPU suite, then C2 / DP / C5 A/B against the variants
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONFAULTHANDLER=1
OUT=${OUT:-gpurun_out/r05b27}
mkdir -p $OUT
V=recommendar-systems_amd/rsx/lib/variants
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $OUT/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed|error" $OUT/pytest_gpu.log | tail -3; [ $rc -eq 0 ] || exit $rc
line() { python -c "import json;d=json.load(open('$OUT/$1.json'));print('$1', round(d['ms_per_step'],4), round(d['value'],1))"; }
for i in 1 2; do
  for v in tagb4 tagb1 tagb8; do
    L=""; [ $v = tagb4 ] || L=$V/$v/librsx.so
    env ${L:+RSX_LIB=$L} timeout -k 10 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline > $OUT/c2_${v}_$i.json 2> $OUT/c2_${v}_$i.err || exit 1
    line c2_${v}_$i
    env ${L:+RSX_LIB=$L} timeout -k 10 300 python bench.py --dp --steps 300 --warmup 30 --no-cpu-baseline > $OUT/dp_${v}_$i.json 2> $OUT/dp_${v}_$i.err || exit 1
    line dp_${v}_$i
  done
done
for v in tagb4 tagb1; do
  L=""; [ $v = tagb4 ] || L=$V/$v/librsx.so
  env ${L:+RSX_LIB=$L} timeout -k 10 300 python bench.py --workload c5 --steps 30 --warmup 6 --no-cpu-baseline > $OUT/c5_$v.json 2> $OUT/c5_$v.err || exit 1
  line c5_$v
done
OUT=$OUT bash tools/gpu/r05_batch26.sh || exit 1
echo done
