# C1 LayerGCN bench: current tree vs oldtree/ (the session-start commit), alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for t in new old new old; do
  if [ $t = new ]; then D=$GRAFT_REPO_ROOT; else D=$GRAFT_REPO_ROOT/oldtree; fi
  (cd $D && timeout -k 10 300 python bench.py --workload c1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/c1_$t.json 2> $GRAFT_REPO_ROOT/gpurun_out/c1_$t.err) || exit 1
  python -c "import json; d=json.load(open('gpurun_out/c1_$t.json')); print('$t', round(d['value']), d['ms_per_step'])"
done
