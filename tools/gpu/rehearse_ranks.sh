# N-rank bench code paths rehearsed on a one-GPU box: every rank on GPU 0 over gloo
# (RSX_BENCH_SAME_DEVICE=1, RSX_BENCH_BACKEND=gloo; RCCL refuses two ranks per GPU).
# Checks the launcher (bench.py --gpus N), the sharded engines and the per-rank report;
# the numbers are not measurements (host-staged collectives, ranks sharing one GPU).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/rehearse}
mkdir -p $OUT
export RSX_BENCH_SAME_DEVICE=1 RSX_BENCH_BACKEND=gloo
[ -n "$SKIP_C2" ] || timeout -k 10 150 python bench.py --gpus 2 --workload c2 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c2_2.json 2> $OUT/c2_2.err || { tail -30 $OUT/c2_2.err; exit 1; }
[ -n "$SKIP_C2" ] || python -c "import json; d=json.load(open('$OUT/c2_2.json')); print('c2 x2', d['n_gpus'], d['value'], [r['ms_per_step'] for r in d['per_rank']])"
timeout -k 10 170 python bench.py --gpus 2 --workload c5 --steps 6 --warmup 6 --no-cpu-baseline > $OUT/c5_2.json 2> $OUT/c5_2.err || { tail -30 $OUT/c5_2.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/c5_2.json')); print('c5 x2', d['n_gpus'], d['value'], d['config']['parallelism'], [r['ms_per_step'] for r in d['per_rank']])"
timeout -k 10 170 python bench.py --gpus 2 --workload c4 --c4-chunks 2 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/c4_2.json 2> $OUT/c4_2.err || { tail -30 $OUT/c4_2.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/c4_2.json')); print('c4 x2', d['n_gpus'], d['value'], [r['ms_per_step'] for r in d['per_rank']])"
