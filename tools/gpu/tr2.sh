# kernel timeline of the sharded engine at one rank (bench --sharded)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/tr2
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr2 -o t -- python bench.py --sharded --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/tr2/b.json 2> gpurun_out/tr2/b.err
rc=$?; echo "rc=$rc"; cat gpurun_out/tr2/b.json; exit $rc
