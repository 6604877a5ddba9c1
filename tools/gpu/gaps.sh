set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/gaps
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/gaps -o c2 -- python bench.py --workload c2 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/gaps/c2.json 2> gpurun_out/gaps/c2.err || exit 1
f=$(find /tmp/gaps -name '*kernel_trace.csv' | head -1)
python tools/gpu/gaps.py "$f" "${1:-sample}" 10 > gpurun_out/gaps/c2_gaps.txt
cat gpurun_out/gaps/c2_gaps.txt
