# SpMM work-block cap sweep on the default C2 bench line: PAIRS of
# RSX_SPMM_MAXB:RSX_SPMM_MAXB_ADAM (the Adam-epilogue kind's own cap)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/maxb}
mkdir -p $OUT
for pr in ${PAIRS:-2048:2048 1536:1024 2048:1024 1536:1280 2048:1280 1536:1536 2048:2048 1536:1024}; do
  m=${pr%%:*}; ma=${pr##*:}
  RSX_SPMM_MAXB=$m RSX_SPMM_MAXB_ADAM=$ma timeout -k 10 200 python bench.py --steps 400 --warmup 40 --no-cpu-baseline > $OUT/b_$m.$ma.json 2> $OUT/b_$m.$ma.err || exit 1
  python -c "import json,sys; d=json.load(open('$OUT/b_$m.$ma.json')); print('$m $ma', round(d['ms_per_step']*1e3,2), 'us/step', [ (k['kernel'][:22], round(k['avg_launch_ms']*1e3,2)) for k in d['roofline_kernels']])"
done
