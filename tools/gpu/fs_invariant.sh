# full-sort screen: the CPU-anchored exactness test on the product library, then on the
# reverted lean variant (tools/fs_lean_variant.py) -- expected to fail on the masked-heavy users
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/fsinv}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_realshape.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "screen_exact" > $OUT/product.log 2>&1
rc=$?; tail -4 $OUT/product.log; [ $rc -eq 0 ] || exit $rc
RSX_LIB=$GRAFT_REPO_ROOT/recommendar-systems_amd/rsx/lib/variants/fs_lean/librsx.so timeout -k 10 600 python -u -m pytest tests/test_gpu_realshape.py tests/test_gpu_kernels.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "screen_exact" > $OUT/lean.log 2>&1
echo "lean variant pytest rc=$?"
grep -E "^FAILED|rows \[|passed|failed" $OUT/lean.log | head -40
