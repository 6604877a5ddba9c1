# rsx_linear_bwd at the C5 projection shape under the plan knobs (RSX_LBWD_IG / RSX_LBWD_WAVES),
# then the C5 / C3 legs at HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/lbwd}
mkdir -p $OUT
for cfg in "2 2048" "1 2048" "4 2048" "2 1024" "2 3072" "1 3072"; do
  set -- $cfg
  RSX_LBWD_IG=$1 RSX_LBWD_WAVES=$2 timeout -k 10 120 python tools/gpu/micro_gemm.py > $OUT/ig$1_w$2.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$OUT/ig$1_w$2.json'));print('ig=$1 waves=$2', round(d['rsx_linear_bwd_ms']*1e3,1), 'us')"
done
for w in c5 c3; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --steps 30 --warmup 6 > $OUT/$w.json 2> $OUT/$w.err || exit 1
  python -c "import json;d=json.load(open('$OUT/$w.json'));print('$w', d['ms_per_step'])"
done
