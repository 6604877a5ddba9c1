# one step of the row-sharded engine at ONE rank (bench --sharded): kernel sequence + line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/shseq}
mkdir -p $OUT
timeout -k 10 300 python bench.py --sharded --no-cpu-baseline --steps 100 --warmup 10 > $OUT/line.json 2> $OUT/line.err || exit 1
python -c "import json;d=json.load(open('$OUT/line.json'));print('sharded 1 rank', d['ms_per_step'])"
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 --warmup 10 > $OUT/line_unsharded.json 2> $OUT/line_u.err || exit 1
python -c "import json;d=json.load(open('$OUT/line_unsharded.json'));print('unsharded', d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/p -o t -- python bench.py --sharded --no-cpu-baseline --steps 30 --warmup 6 > $OUT/b.json 2> $OUT/b.err || exit 1
f=$(find $OUT/p -name '*kernel_trace.csv' | head -1)
python tools/seq_trace.py "$f" ${ANCHOR:-bpr} 40 > $OUT/seq.txt || true
python tools/seq_trace.py "$f" ${ANCHOR:-bpr} 41 > $OUT/seq2.txt || true
rm -f "$f"
tail -1 $OUT/seq.txt
