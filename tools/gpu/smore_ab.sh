# SMORE GPU tests, then the C5 / C3 bench lines and one step's kernel sequence of each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/ab}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_smore.py tests/test_gpu_smore_fuse.py tests/test_gpu_smore_dist.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for w in c5 c3; do
  for v in ${VARIANTS:-1}; do
    RSX_SMORE_WGRAD_STREAM=$v timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --steps 30 --warmup 6 > $OUT/${w}_w$v.json 2> $OUT/${w}_w$v.err || exit 1
    python -c "import json;d=json.load(open('$OUT/${w}_w$v.json'));print('$w wgrad-stream=$v', d['ms_per_step'])"
  done
done
OUT=$OUT/seq bash tools/gpu/c5_seq.sh
LEG=c3 OUT=$OUT/seq3 bash tools/gpu/c5_seq.sh
