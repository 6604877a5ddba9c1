# A/B of the bench step: current librsx vs rsx/lib/variants/$1 (alternating, twice each)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
V=$1
for v in base $V base $V; do
  if [ $v = base ]; then L=$PWD/recommendar-systems_amd/rsx/lib/librsx.so; else L=$PWD/recommendar-systems_amd/rsx/lib/variants/$v/librsx.so; fi
  RSX_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab_$v.json')); print('$v', round(d['ms_per_step']*1000,2), 'us/step', round(d['fullsort']['s_per_eval']*1e3,3), 'ms/eval')"
done
