# FETCH / WRITE PMC passes (separate runs) of spmm_main<256, *> in C4's one-rank share,
# with a heartbeat file so the long host-side graph build is not taken for a hang
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/c4pmc}
mkdir -p $OUT
A="--workload c4 --c4-chunks 1 --steps 3 --warmup 1 --no-cpu-baseline --eval-users 4096"
beat() { while kill -0 $1 2>/dev/null; do date +%s >> $OUT/heartbeat; sleep 20; done; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 600 rocprofv3 --pmc $c --kernel-include-regex "spmm_main<256" --output-format csv -d $OUT/pmc_$c -o run -- python bench.py $A > $OUT/pmc_$c.json 2> $OUT/pmc_$c.err &
  pid=$!
  beat $pid &
  wait $pid || { tail -20 $OUT/pmc_$c.err; exit 1; }
done
echo done
