# round 6: nce_bwd_t at d = 64 (RSX_NCE_T64=1): the InfoNCE tests and the SMORE fixture tests with
# it, then the C3 line with it off and on
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/r06nce64}
mkdir -p "$OUT"
RSX_NCE_T64=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_smore_fuse.py tests/test_gpu_smore.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -60 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for T in 0 1 0 1; do
  RSX_NCE_T64=$T timeout -k 10 300 python bench.py --workload c3 --steps 30 --warmup 6 --no-cpu-baseline \
    > "$OUT/c3_t$T.json" 2> "$OUT/c3_t$T.err" || { tail -20 "$OUT/c3_t$T.err"; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/c3_t$T.json'))
k=[r for r in d['roofline_kernels'] if 'nce' in r['kernel']][0]
print('c3 t64=$T', round(d['ms_per_step'],4), 'nce', round(k['avg_launch_ms']*1e3,1), 'us', round(k['frac'],3))"
done
echo done
