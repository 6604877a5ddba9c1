set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ps
for cfg in "512 512" "1536 512" "2048 256" "4096 128"; do
  set -- $cfg
  for w in c3 c5; do
    RSX_PROJ_TARGET=$1 RSX_PROJ_MINK=$2 timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --steps 30 --warmup 6 > gpurun_out/ps/$w.json 2>/dev/null || exit 1
    echo "$cfg $w $(python -c "import json;print(round(json.load(open('gpurun_out/ps/$w.json'))['ms_per_step'],3))")"
  done
done
