set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/p1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p1 -o t -- python3 bench.py --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/p1/bench.json 2> gpurun_out/p1/bench.err || exit 1
