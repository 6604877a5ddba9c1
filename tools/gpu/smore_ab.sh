# C3 / C5 step time: the batch-row preference forward split (RSX_PREF_SPLIT) x the two
# projections' backward on two streams (RSX_PROJ_STREAM)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=${OUT:-gpurun_out/sab}
mkdir -p $OUT
for w in c3 c5; do
  for sp in 0 1; do
    for ps in 0 1; do
      RSX_PREF_SPLIT=$sp RSX_PROJ_STREAM=$ps timeout -k 10 200 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > $OUT/${w}_s${sp}_p${ps}.json 2> $OUT/${w}_s${sp}_p${ps}.err || exit 1
      python -c "import json; d=json.load(open('$OUT/${w}_s${sp}_p${ps}.json')); print('$w split=$sp proj_stream=$ps', round(d['ms_per_step'], 3))"
    done
  done
done
