# the fused-round sharded step: its GPU tests, the one-rank RCCL sharded engine (bench
# --sharded) fused vs one exchange per layer, and the 2-rank gloo rehearsal of c2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/fused}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_sharded_trainer.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; tail -15 $OUT/pytest.log | grep -v "^$"; [ $rc -eq 0 ] || exit $rc
for f in 1 0; do
  RSX_SHARDED_FUSED=$f timeout -k 10 200 python bench.py --sharded --steps 200 --warmup 20 --no-cpu-baseline > $OUT/sharded_f$f.json 2> $OUT/sharded_f$f.err || { tail -20 $OUT/sharded_f$f.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/sharded_f$f.json')); print('fused=$f', d['ms_per_step'], d['value'], d['config'].get('parallelism'))"
done
SKIP_C4=1 OUT=$OUT/rehearse timeout -k 10 400 bash tools/gpu/rehearse_ranks.sh 2>&1 | head -3
