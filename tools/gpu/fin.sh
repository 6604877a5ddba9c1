# final profile set of the round: kernel-trace stats of the bench, then the full bench line (with the CPU baseline)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r12
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r12/stats -o bench -- python bench.py --no-cpu-baseline > gpurun_out/r12/bench_prof.json 2> gpurun_out/r12/bench_prof.err && \
timeout -k 10 600 python bench.py > gpurun_out/r12/bench_full.json 2> gpurun_out/r12/bench_full.err
rc=$?
find gpurun_out/r12 -name '*kernel_trace.csv' -delete
echo "rc=$rc"
exit $rc
