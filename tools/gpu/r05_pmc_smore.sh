# round 5: counter passes for the SMORE kernels furthest below their
# roofline at C5 — the batch-row preference backward (pref_bwd_rows<128>, pref_segsum),
# the weight gradients (wgrad_part<128>) and the InfoNCE backward (nce_bwd_t<128>) — plus
# the projections' backward (linear_bwd) for reference: issue / wait split, VALU / LDS /
# MFMA busy, LDS bank conflicts, L2-miss bytes.  One pass per counter group (rocprofv3
# does not split passes), each under its own kill timer.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r05pmc}
mkdir -p $OUT
A="--workload c5 --steps 4 --warmup 2 --no-cpu-baseline"
RX=${RX:-"pref_bwd_rows|wgrad_part|nce_bwd_t|pref_segsum|linear_bwd|gates_bwd_res|spec_bwd"}
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
pass() {  # name, counters
  local name=$1; shift
  timeout -s KILL 300 rocprofv3 --pmc "$@" --kernel-include-regex "$RX" --output-format csv -d $OUT/$name -o run \
    -- python bench.py $A > $OUT/$name.line 2> $OUT/$name.err || { tail -5 $OUT/$name.err; return 1; }
  echo "$name ok"
}
pass p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS || exit 1
pass p2 SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM || exit 1
pass p3 FETCH_SIZE || exit 1
pass p4 WRITE_SIZE || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --kernel-include-regex "$RX" --output-format csv -d $OUT/kt -o run \
  -- python bench.py $A > $OUT/kt.line 2> $OUT/kt.err || exit 1
echo done
