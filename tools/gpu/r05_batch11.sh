# round 5, eleventh GPU batch: the compact-rows SMORE loss backward in one launch and the compact-rows BPR variant (RSX_BPR_SMORE_ROWS: gradient rows stored, no zero fill)
# (rsx_smore_loss_rows_bwd: InfoNCE rows stored, negatives' rows zeroed, BPR rows scaled);
# the SMORE GPU tests, the C5 / C3 lines, one C5 step's exclusive-time breakdown
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONFAULTHANDLER=1
OUT=${OUT:-gpurun_out/r05b11}
mkdir -p $OUT
timeout -k 10 800 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_smore.py tests/test_gpu_smore_fuse.py tests/test_gpu_e2e.py tests/test_gpu_smore_dist.py \
  -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" $OUT/pytest.log | tail -12; [ $rc -eq 0 ] || exit $rc
for w in c5 c3; do
  timeout -k 10 300 python bench.py --workload $w --steps 30 --warmup 6 --no-cpu-baseline > $OUT/$w.json 2> $OUT/$w.err || exit 1
  python -c "import json;d=json.load(open('$OUT/$w.json'));print('$w', d['ms_per_step'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/c5t -o t -- \
  python3 bench.py --workload c5 --steps 12 --warmup 6 --no-cpu-baseline > $OUT/c5t.json 2> $OUT/c5t.err \
  || { tail -20 $OUT/c5t.err; exit 1; }
python tools/exposed.py $OUT/c5t/t_kernel_trace.csv adam_multi 2 40 > $OUT/c5_exposed.txt && head -24 $OUT/c5_exposed.txt
echo done
