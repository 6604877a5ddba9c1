# one C2 step's kernel timeline under rocprofv3 --kernel-trace, for each env setting in $VARIANTS
# (e.g. VARIANTS="RSX_BATCH_LIST=1 RSX_BATCH_LIST=0")
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/steptl}
mkdir -p $OUT
i=0
for v in ${VARIANTS:-X=1}; do
  i=$((i+1))
  export $v
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/p$i -o t -- python bench.py --no-cpu-baseline --steps 60 --warmup 10 ${BENCH_ARGS} > $OUT/b$i.json 2> $OUT/b$i.err || { tail -20 $OUT/b$i.err; exit 1; }
  f=$(find $OUT/p$i -name '*kernel_trace.csv' | head -1)
  echo "== $v"; python tools/steptrace.py "$f" ${ANCHOR:-bpr_fused} 40 ${BACK:-4} | tee $OUT/tl$i.txt
  rm -f "$f"
done
