# kernel timeline of the C1 (LayerGCN) bench step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/tr3
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr3 -o t -- python bench.py --workload c1 --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/tr3/b.json 2> gpurun_out/tr3/b.err
rc=$?; echo "rc=$rc"; exit $rc
