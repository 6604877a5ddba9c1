# round 4: the data-parallel LightGCN step (rsx.dp / csrc/dp.hip) and the changed paths:
# the DP / dist / sampler GPU tests, then the DP engine at one rank (bench --dp), a
# 2-rank same-GPU rehearsal over gloo, and the default line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r04dp}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; tail -15 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 > $OUT/c2.json 2> $OUT/c2.err || { tail -20 $OUT/c2.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 --dp > $OUT/c2_dp1.json 2> $OUT/c2_dp1.err || { tail -20 $OUT/c2_dp1.err; exit 1; }
RSX_BENCH_SAME_DEVICE=1 RSX_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --no-cpu-baseline --steps 20 --warmup 3 > $OUT/c2_dp2_rehearsal.json 2> $OUT/c2_dp2_rehearsal.err || { tail -20 $OUT/c2_dp2_rehearsal.err; exit 1; }
timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline --steps 30 --warmup 6 > $OUT/c5.json 2> $OUT/c5.err || { tail -20 $OUT/c5.err; exit 1; }
python - <<'PY'
import json
for f in ("c2", "c2_dp1", "c2_dp2_rehearsal", "c5"):
    d = json.load(open(f"gpurun_out/r04dp/{f}.json"))
    print(f, d["value"], d["ms_per_step"], d["config"]["parallelism"], d.get("train_loss_mean"))
PY
