# one C5 (or LEG) step's kernel sequence with queue ids at HEAD (tools/seq_trace.py), plus kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/c5seq}
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p -o t -- python bench.py --workload ${LEG:-c5} --no-cpu-baseline --steps ${STEPS:-20} --warmup 6 > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
f=$(find $OUT/p -name '*kernel_trace.csv' | head -1)
python tools/seq_trace.py "$f" ${ANCHOR:-adam_multi} ${NTH:-12} > $OUT/seq.txt
python tools/seq_trace.py "$f" ${ANCHOR:-adam_multi} $(( ${NTH:-12} + 1 )) > $OUT/seq2.txt
tail -1 $OUT/seq.txt; tail -1 $OUT/seq2.txt
rm -f "$f"
python -c "import json;d=json.load(open('$OUT/b.json'));print(d['ms_per_step'])"
