# round 4, batch E: C4 at the modelled 8-rank job with the SpMM work-block cap lowered (CUs
# left free for the collectives' workgroups), then the N = 1 anchor (the full 10M-user graph)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r04e}
mkdir -p $OUT
A="--workload c4 --steps 8 --warmup 2 --no-cpu-baseline --eval-users 4096"
for mb in 1536 1024; do
  RSX_COMM_SIM=8 RSX_SPMM_MAXB=$mb timeout -k 10 500 python bench.py $A > $OUT/sim_w8_maxb$mb.json 2> $OUT/sim_w8_maxb$mb.err || { tail -5 $OUT/sim_w8_maxb$mb.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/sim_w8_maxb$mb.json')); print('maxb $mb', round(d['ms_per_step'], 3))"
done
RSX_SPMM_MAXB=1536 timeout -k 10 500 python bench.py $A --c4-chunks 1 --batch 256 > $OUT/compute_w8_maxb1536.json 2> $OUT/c.err || exit 1
python -c "import json; d=json.load(open('$OUT/compute_w8_maxb1536.json')); print('compute maxb 1536', round(d['ms_per_step'], 3))"
OUT=$OUT PART=2 bash tools/gpu/r04_c4.sh
