# round 6: the `bench.py --gpus N` default at N > 1 (C4-d64, row-sharded) rehearsed through its
# own launcher with 2 ranks sharing the box's one GPU over gloo (RCCL refuses two ranks on one
# GPU; the real N-GPU run is the driver's), and data-parallel SMORE (C5) the same way
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/r06reh}
mkdir -p "$OUT"
export RSX_BENCH_SAME_DEVICE=1 RSX_BENCH_BACKEND=gloo
timeout -k 10 900 python bench.py --gpus 2 --steps 3 --warmup 1 --eval-users 1024 > "$OUT/default_n2.json" 2> "$OUT/default_n2.err" || { tail -30 "$OUT/default_n2.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/default_n2.json')); print('default n2', d['config']['workload'][:40], d['n_gpus'], d['value'], d['ms_per_step'], d['config']['parallelism'], [r['ms_per_step'] for r in d['per_rank']])"
timeout -k 10 900 python bench.py --gpus 2 --workload c5 --steps 4 --warmup 2 > "$OUT/c5_n2.json" 2> "$OUT/c5_n2.err" || { tail -30 "$OUT/c5_n2.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/c5_n2.json')); print('c5 n2', d['n_gpus'], d['value'], d['ms_per_step'], d['config']['parallelism'])"
echo done
