# rsx_linear_bwd tuning sweep (IG x target waves) on the C3 / C5 legs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/lb
for cfg in "2 2048" "4 2048" "2 4096" "1 4096" "2 1024"; do
  set -- $cfg
  for w in c3 c5; do
    RSX_LBWD_IG=$1 RSX_LBWD_WAVES=$2 timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --steps 30 --warmup 6 > gpurun_out/lb/$w.json 2>/dev/null || exit 1
    echo "$cfg $w $(python -c "import json;print(round(json.load(open('gpurun_out/lb/$w.json'))['ms_per_step'],3))")"
  done
done
