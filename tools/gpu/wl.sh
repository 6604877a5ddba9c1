# the other configs' bench lines (C1 LayerGCN baby, C3 SMORE baby, C5 SMORE clothing d=128)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for w in c1 c3 c5; do
  timeout -k 10 400 python bench.py --workload $w --no-cpu-baseline > gpurun_out/wl_$w.json 2> gpurun_out/wl_$w.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/wl_$w.json')); print('$w', round(d['value']), d['ms_per_step'], d.get('fullsort_items_per_s'))"
done
