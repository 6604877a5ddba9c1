# price the batch-row preference backward's float atomics: C5 with a plain-store variant
# (timing only: wrong where rows repeat) against the product library
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pa}
mkdir -p $OUT
V=recommendar-systems_amd/rsx/lib/variants/plainst/librsx.so
RSX_LIB=$V timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/v -o v -- python bench.py --workload c5 --no-cpu-baseline --steps 20 --warmup 6 > $OUT/v.json 2> $OUT/v.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p -o p -- python bench.py --workload c5 --no-cpu-baseline --steps 20 --warmup 6 > $OUT/p.json 2> $OUT/p.err || exit 1
find $OUT -name '*kernel_trace.csv' -delete
for x in v p; do f=$(find $OUT/$x -name '*kernel_stats.csv' | head -1); grep pref_bwd_rows "$f" | cut -d, -f1-4; done
