# round 4: the data-parallel LightGCN leg (rsx.dp, csrc/dp.hip) measured at one rank over
# a real one-rank RCCL communicator (graph-captured), beside the single-GPU engine, plus
# its kernel sequence; the N-rank model in DESIGN.md §6.1 starts from these
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export OUT=${OUT:-gpurun_out/r04dpm}
mkdir -p $OUT
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 300 > $OUT/c2.json 2> $OUT/c2.err || { tail -20 $OUT/c2.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 300 --dp > $OUT/c2_dp1.json 2> $OUT/c2_dp1.err || { tail -20 $OUT/c2_dp1.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_dp1 -o dp1 -- python bench.py --no-cpu-baseline --steps 100 --dp > $OUT/c2_dp1_prof.json 2> $OUT/c2_dp1_prof.err || exit 1
find $OUT -name '*kernel_trace.csv' -delete
python - <<'PY'
import json, os
for f in ("c2", "c2_dp1", "c2_dp1_prof"):
    d = json.load(open(os.path.join(os.environ.get("OUT", "gpurun_out/r04dpm"), f + ".json")))
    print(f, round(d["value"] / 1e6, 3), "M/s", round(d["ms_per_step"], 4), "ms", d["config"]["parallelism"])
PY
