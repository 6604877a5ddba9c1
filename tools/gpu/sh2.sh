set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/psh
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/psh -o sh -- python3 bench.py --sharded --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/psh/bench.json 2> gpurun_out/psh/bench.err || exit 1
cat gpurun_out/psh/bench.json | cut -c1-400
find gpurun_out/psh -name '*.csv' | head
