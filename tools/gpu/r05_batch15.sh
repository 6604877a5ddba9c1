# round 5, fifteenth GPU batch: the SMORE batch rows and their tags in one launch (rsx_batch_rows),
# the re-tags as one launch each (rsx_tag_rows_next);
# the SMORE GPU tests, the C5 / C3 lines, one C5 step's exclusive-time breakdown
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONFAULTHANDLER=1
OUT=${OUT:-gpurun_out/r05b15}
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
