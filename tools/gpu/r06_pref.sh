# round 6: the preference block (saved activations, occurrence plan) -- its unit tests and the SMORE
# fixture tests, then the C3 / C5 lines (no CPU baseline) with the paired projection backward on and off
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/r06pref}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_smore_fuse.py tests/test_gpu_smore.py -m gpu -x -v --timeout 300 \
  --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -60 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for W in c3 c5; do
  for S in 1 0; do  # RSX_LBWD_PAIR on / off
    RSX_LBWD_PAIR=$S timeout -k 10 300 python bench.py --workload $W --steps 60 --warmup 6 --no-cpu-baseline \
      > "$OUT/${W}_pair$S.json" 2> "$OUT/${W}_pair$S.err" || { tail -20 "$OUT/${W}_pair$S.err"; exit 1; }
    python -c "
import json; d=json.load(open('$OUT/${W}_pair$S.json'))
k=[r for r in d['roofline_kernels'] if 'pref_rows' in r['kernel']][0]
print('$W pair=$S', round(d['ms_per_step'],4), 'pref', round(k['avg_launch_ms']*1e3,1), 'us', round(k['frac'],3))"
  done
done
echo done
