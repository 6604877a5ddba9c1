# C4 at a modelled W-rank job (RSX_COMM_SIM=W, one rank's share on one GPU): the kernel
# sequence of one step period (BPR to BPR) with queue ids, so the comm stream's injected
# collectives (sim_collective) can be read against the compute stream's products
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
W=${W:-8}
OUT=${OUT:-gpurun_out/c4trace_w$W}
mkdir -p $OUT
RSX_COMM_SIM=$W timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/p -o t -- python bench.py --workload c4 --steps 4 --warmup 2 --no-cpu-baseline --eval-users 1024 > $OUT/b.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 1; }
f=$(find $OUT/p -name '*kernel_trace.csv' | head -1)
python tools/seq_trace.py "$f" bpr_fused 3 > $OUT/seq.txt || true
python tools/seq_trace.py "$f" bpr_fused 4 > $OUT/seq2.txt || true
rm -f "$f"
tail -1 $OUT/seq.txt
