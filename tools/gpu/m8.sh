set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in base g16 w6 pf0 base g16 w6 pf0; do
  if [ $v = base ]; then L=recommendar-systems_amd/rsx/lib/librsx.so; else L=recommendar-systems_amd/rsx/lib/variants/$v/librsx.so; fi
  RSX_LIB=$PWD/$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 400 > gpurun_out/var_$v.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/var_$v.json')); print('$v', round(d['value']/1e6,3), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms']*1e3,2), round(d['fullsort']['s_per_eval']*1e3,3))"
done
