set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu/fs_dr.sh > gpurun_out/fsdr.txt 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_smore.py tests/test_gpu_smore_fuse.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/smore_tests.txt 2>&1 || exit 1
timeout -k 10 200 python bench.py --workload c5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/c5b.json 2> gpurun_out/c5b.err || exit 1
timeout -k 10 200 python bench.py --workload c3 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/c3b.json 2> gpurun_out/c3b.err
