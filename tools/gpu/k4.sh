# K = 4 (the reference's LightGCN.yaml default): the tests that cover the stored-layer
# step at K = 4, then C2-shaped bench lines at K = 4 with batch-row tags (stored layers)
# and without (the dense path), and the default K = 3 line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/k4}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_realshape.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "tags or hub_graph or nan_loss or layergcn_c_step" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for cfg in "4 1" "4 0" "3 1"; do
  set -- $cfg
  RSX_BATCH_TAGS=$2 timeout -k 10 300 python bench.py --n-layers $1 --steps 200 --warmup 20 --no-cpu-baseline > $OUT/c2_k$1_t$2.json 2> $OUT/c2_k$1_t$2.err || { tail -20 $OUT/c2_k$1_t$2.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/c2_k$1_t$2.json')); print('K=$1 tags=$2', round(d['value']), round(d['ms_per_step'], 4))"
done
