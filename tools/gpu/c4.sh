set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/c4
timeout -k 10 1000 python bench.py --workload c4 --steps 6 --warmup 2 > gpurun_out/c4/c4_full.json 2> gpurun_out/c4/c4_full.err || { tail -20 gpurun_out/c4/c4_full.err; exit 1; }
cat gpurun_out/c4/c4_full.json
