# round 6: LDS bank conflicts of the InfoNCE backward after the D + 8
# padding of its reduction tile (C5, nce_bwd_t<128, 2>; C3, nce_bwd<64>), one counter pass each
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/r06pmc}
mkdir -p "$OUT"
for W in c5 c3; do
  timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES \
    --kernel-include-regex "nce_bwd|pref_bwd_rows|gates_bwd_res" --output-format csv -d "$OUT/$W" -o run \
    -- python bench.py --workload $W --steps 4 --warmup 2 --no-cpu-baseline > "$OUT/$W.line" 2> "$OUT/$W.err" || { tail -5 "$OUT/$W.err"; exit 1; }
  echo "$W pmc ok"
done
echo done
