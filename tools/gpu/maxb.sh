set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -x -p no:cacheprovider -k "spmm or forward or fused" 2>&1 | tail -2 || exit 1
for m in 1024 1536 2048 3072 100000; do
  RSX_SPMM_MAXB=$m timeout -k 10 100 python tools/gpu/micro.py spmmx > gpurun_out/mx_$m.txt || exit 1
  RSX_SPMM_MAXB=$m timeout -k 10 200 python bench.py --no-cpu-baseline --steps 400 > gpurun_out/mb_$m.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/mb_$m.json')); print('$m', round(d['value']/1e6,3), round(d['ms_per_step'],4), open('gpurun_out/mx_$m.txt').read().strip())"
done
