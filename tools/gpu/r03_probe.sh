# fs_screen vs user count (segmentation onset) with and without the balanced split, and
# one C5 step's kernel sequence (tools/seq_trace.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/probe
mkdir -p $O
(echo "default"; timeout -k 10 120 python tools/gpu/fsbal.py 32768 33024 34000 35598 40960 49152 65536 && echo "RSX_FS_SEG=0"; RSX_FS_SEG=0 timeout -k 10 120 python tools/gpu/fsbal.py 32768 33024 34000 35598 40960 49152 65536) > $O/fs_curve.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/p -o t -- python bench.py --workload c5 --no-cpu-baseline --steps 12 --warmup 4 > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
f=$(find $O/p -name '*kernel_trace.csv' | head -1)
python tools/seq_trace.py "$f" adam_multi 8 > $O/c5_seq.txt
rm -f "$f"
