# round 6: C2 under a node relabelling (RSX_BENCH_RELABEL: degree / rcm)
# against the plain order: the bench line (step time, STORE / ADAM layer times) and the
# PMC FETCH_SIZE / WRITE_SIZE of the STORE (<64, 0>) and ADAM (<64, 3>) launches, separate passes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/r06rl}
mkdir -p "$OUT"
for R in none degree rcm; do
  E="RSX_X=0"; [ "$R" != none ] && E="RSX_BENCH_RELABEL=$R"
  timeout -k 10 300 env $E python bench.py --steps 300 --warmup 30 --no-cpu-baseline > "$OUT/line_$R.json" 2> "$OUT/line_$R.err" || { tail -20 "$OUT/line_$R.err"; exit 1; }
  python -c "
import json; d = json.load(open('$OUT/line_$R.json'))
print('$R', round(d['ms_per_step'], 4), 'ms/step', {k['kernel'][:22]: round(k['avg_launch_ms'] * 1e3, 1) for k in d['roofline_kernels']})"
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 env $E rocprofv3 --pmc $C --kernel-include-regex "spmm_main<64, [03]>" --output-format csv \
      -d "$OUT/pmc_${R}_$C" -o run -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline > /dev/null 2> "$OUT/pmc_${R}_$C.err" || { tail -5 "$OUT/pmc_${R}_$C.err"; exit 1; }
  done
done
echo done
