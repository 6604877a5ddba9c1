# kernel timeline of the bench step (kernel trace kept for tools/steptrace.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/tr
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr -o t -- python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/tr/b.json 2> gpurun_out/tr/b.err
rc=$?; echo "rc=$rc"; exit $rc
