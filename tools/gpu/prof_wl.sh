set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pw
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pw/c1 -o c1 -- python bench.py --workload c1 --steps 100 --warmup 10 > gpurun_out/pw/c1.json 2> gpurun_out/pw/c1.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pw/c5 -o c5 -- python bench.py --workload c5 --steps 20 --warmup 3 > gpurun_out/pw/c5.json 2> gpurun_out/pw/c5.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pw/c3 -o c3 -- python bench.py --workload c3 --steps 20 --warmup 3 > gpurun_out/pw/c3.json 2> gpurun_out/pw/c3.err || exit 1
find gpurun_out/pw -name '*kernel_trace.csv' -delete
