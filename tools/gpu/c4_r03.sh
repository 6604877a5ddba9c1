# C4 one rank's 1/8 share on one GPU (1.25M users x 1M items, d = 256, the sharded
# engine at one rank: the sparse exchange schedule), round 3: the line with the CPU
# baseline, the dense schedule's line, rocprofv3 kernel stats, FETCH / WRITE PMC passes
# of spmm_main<256, *>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/c4r3}
mkdir -p $OUT
A="--workload c4 --c4-chunks 1"
timeout -k 10 500 python bench.py $A --steps 10 --warmup 2 --cpu-budget 20 > $OUT/c4_one_rank.json 2> $OUT/c4_one_rank.err || { tail -20 $OUT/c4_one_rank.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/c4_one_rank.json')); print('sparse', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['cpu_baseline'])"
RSX_SPARSE_MIN_BYTES=1000000000000 timeout -k 10 400 python bench.py $A --steps 10 --warmup 2 --no-cpu-baseline > $OUT/c4_one_rank_dense.json 2> $OUT/c4_one_rank_dense.err || { tail -20 $OUT/c4_one_rank_dense.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/c4_one_rank_dense.json')); print('dense', d['value'], d['ms_per_step'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o c4 -- python bench.py $A --steps 10 --warmup 2 --no-cpu-baseline > $OUT/c4_prof.json 2> $OUT/c4_prof.err || { tail -20 $OUT/c4_prof.err; exit 1; }
find $OUT -name '*kernel_trace.csv' -delete
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "spmm_main<256" --output-format csv -d $OUT/pmc_fetch -o run -- python bench.py $A --steps 4 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/pmc_fetch.err || { tail -20 $OUT/pmc_fetch.err; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "spmm_main<256" --output-format csv -d $OUT/pmc_write -o run -- python bench.py $A --steps 4 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/pmc_write.err || { tail -20 $OUT/pmc_write.err; exit 1; }
echo done
