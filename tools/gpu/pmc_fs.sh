# SQ counters of the screened full-sort kernel (fs_screen<64>) on tools/gpu/fsbal.py
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmcfs}
mkdir -p $OUT
for m in ${MODES:-0 5}; do
  RSX_FS_MODE=$m timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES \
    --kernel-include-regex "fs_screen" --output-format csv -d $OUT/m$m -o run -- python tools/gpu/fsbal.py ${NBS:-32768} > $OUT/m$m.log 2>&1 || exit 1
done
python - <<'PY'
import csv, glob, os, collections
out = os.environ.get("OUT", "gpurun_out/pmcfs")
for f in sorted(glob.glob(out + "/m*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(f)
    for k in sorted(acc): print(f"  {k}: {acc[k] / max(1, n[k]) * 1:.4g} (per dispatch avg over {n[k]} rows)")
PY
