set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/wl
timeout -k 10 300 python bench.py --workload c1 --steps 100 --warmup 10 > gpurun_out/wl/c1.json 2> gpurun_out/wl/c1.err && cat gpurun_out/wl/c1.json && \
timeout -k 10 400 python bench.py --workload c3 --steps 30 --warmup 5 > gpurun_out/wl/c3.json 2> gpurun_out/wl/c3.err && cat gpurun_out/wl/c3.json && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/wl/prof_c3 -o c3 -- python bench.py --workload c3 --steps 30 --warmup 5 > gpurun_out/wl/c3p.json 2> gpurun_out/wl/c3p.err
echo "rc=$?"
