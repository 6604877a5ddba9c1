# kernel trace of one bench leg, summarised per step period (tools/trace_gaps.py): LEG=c3 ANCHOR=adam_multi
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/tl}
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/p -o t -- python bench.py --workload ${LEG:-c3} --no-cpu-baseline --steps ${STEPS:-30} --warmup 6 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
f=$(find $OUT/p -name '*kernel_trace.csv' | head -1)
python tools/trace_gaps.py "$f" "${ANCHOR:-adam_multi}" ${PERIODS:-12} 45 | tee $OUT/gaps.txt
rm -f "$f"
