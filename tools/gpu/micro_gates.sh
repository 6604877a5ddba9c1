# gates kernels alone: time, then two SQ counter passes on gates_bwd
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/mg}
mkdir -p $OUT
timeout -k 10 120 python tools/gpu/micro_gates.py > $OUT/t.txt 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES \
  --kernel-include-regex "gates_bwd" --output-format csv -d $OUT/a -o run -- python tools/gpu/micro_gates.py > $OUT/a.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD \
  --kernel-include-regex "gates_bwd" --output-format csv -d $OUT/b -o run -- python tools/gpu/micro_gates.py > $OUT/b.log 2>&1
python - <<'PY'
import csv, glob, os, collections
out = os.environ.get("OUT", "gpurun_out/mg")
for f in sorted(glob.glob(out + "/[ab]/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(f)
    for k in sorted(acc): print(f"  {k}: {acc[k] / max(1, n[k]):.4g} per dispatch")
PY
cat $OUT/t.txt; tail -3 $OUT/b.log
