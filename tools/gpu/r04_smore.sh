# round 4: SMORE kernel changes (sorted per-row sums of the preference backward, InfoNCE
# backward on transposed row tiles): the SMORE GPU tests, then the C5 / C3 lines and
# C5's kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r04s}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_smore_fuse.py tests/test_gpu_smore.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for w in c5 c3; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --steps 30 --warmup 6 > $OUT/$w.json 2> $OUT/$w.err || { tail -20 $OUT/$w.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$w.json'));print('$w', d['ms_per_step'], [(r['kernel'][:40], round(r['frac'],3), round(1e3*r['avg_launch_ms'],1)) for r in d.get('roofline_kernels', [])])"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_c5 -o c5 -- python bench.py --workload c5 --no-cpu-baseline --steps 20 --warmup 6 > $OUT/c5_under_rocprof.json 2> $OUT/c5_prof.err || exit 1
find $OUT -name '*kernel_trace.csv' -delete
echo done
