# SMORE GPU tests then one C5 step's kernel sequence (tools/gpu/c5_seq.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/sc}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_smore.py tests/test_gpu_smore_fuse.py tests/test_gpu_smore_dist.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
OUT=$OUT/seq bash tools/gpu/c5_seq.sh
timeout -k 10 300 python bench.py --workload c3 --no-cpu-baseline --steps 30 --warmup 6 > gpurun_out/sc/c3.json 2> gpurun_out/sc/c3.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/sc/c3.json'));print('c3', d['ms_per_step'])"
timeout -k 10 120 python tools/gpu/micro_gemm.py > gpurun_out/sc/micro_gemm.json 2>&1; cat gpurun_out/sc/micro_gemm.json
