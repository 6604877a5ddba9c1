# round 5, eighteenth GPU batch: forward-only weight stagings padded to D + 8 (conflict-free ds_read_b128 in mv_p: gates_fwd, pref_fwd(_rows), the item pass gates)
# ; the SMORE GPU tests, the projection micro-benchmark, the C5 / C3 lines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONFAULTHANDLER=1
OUT=${OUT:-gpurun_out/r05b18}
mkdir -p $OUT
timeout -k 10 800 python -u -m pytest tests/test_gpu_smore.py tests/test_gpu_smore_fuse.py tests/test_gpu_e2e.py \
  -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" $OUT/pytest.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/gpu/micro_gemm.py > $OUT/micro_gemm.json 2> $OUT/micro_gemm.err || exit 1
python -c "import json;d=json.load(open('$OUT/micro_gemm.json'));print('linear_bwd', round(d['rsx_linear_bwd_ms']*1e3,1), 'us')"
for w in c5 c3; do
  timeout -k 10 300 python bench.py --workload $w --steps 30 --warmup 6 --no-cpu-baseline > $OUT/$w.json 2> $OUT/$w.err || exit 1
  python -c "import json;d=json.load(open('$OUT/$w.json'));print('$w', d['ms_per_step'])"
done
echo done
