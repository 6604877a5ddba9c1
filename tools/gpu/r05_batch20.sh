# round 5, twentieth GPU batch: the C4 leg at W = 8 (latency-injected rank 0 share, and
# the share's compute alone) at the final HEAD -- the line's STORE roofline now carries the
# measured PMC fetch traffic of the 1/8-share product launches
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05b20}
mkdir -p $OUT
A="--workload c4 --steps 8 --warmup 2 --no-cpu-baseline --eval-users 4096"
timeout -k 10 500 env RSX_COMM_SIM=8 python bench.py $A > $OUT/sim_w8.json 2> $OUT/sim_w8.err || { tail -20 $OUT/sim_w8.err; exit 1; }
timeout -k 10 500 env RSX_X=0 python bench.py $A --c4-chunks 1 --batch 256 > $OUT/compute_w8.json 2> $OUT/compute_w8.err || { tail -20 $OUT/compute_w8.err; exit 1; }
for n in sim_w8 compute_w8; do
  python -c "import json;d=json.load(open('$OUT/$n.json'));r=d['roofline'];print('$n', round(d['ms_per_step'],3), 'frac', round(r['frac'],3), 'traffic', r.get('traffic'), 'alg', r.get('algorithmic_bytes_per_launch'))"
done
echo done
