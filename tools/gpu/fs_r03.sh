# fs_screen at the sports shape: time per ablation mode (0 full, 5 pass 1 only, 6 no exact
# dots) and SQ counters per mode (two passes of 8 SQ counters each)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/fs_r03}
mkdir -p $OUT
for m in 0 5 6; do
  echo "mode $m" >> $OUT/t.txt
  RSX_FS_MODE=$m timeout -k 10 120 python tools/gpu/fsbal.py 35598 >> $OUT/t.txt 2>&1 || exit 1
done
for m in ${MODES:-0 5}; do
  RSX_FS_MODE=$m timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES \
    --kernel-include-regex "fs_screen" --output-format csv -d $OUT/a$m -o run -- python tools/gpu/fsbal.py 35598 > $OUT/a$m.log 2>&1 || exit 1
  RSX_FS_MODE=$m timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM \
    --kernel-include-regex "fs_screen" --output-format csv -d $OUT/b$m -o run -- python tools/gpu/fsbal.py 35598 > $OUT/b$m.log 2>&1 || exit 1
done
python - <<'PY'
import csv, glob, os, collections
out = os.environ.get("OUT", "gpurun_out/fs_r03")
for f in sorted(glob.glob(out + "/[ab]*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(f)
    for k in sorted(acc): print(f"  {k}: {acc[k] / max(1, n[k]) * 1:.4g} (per dispatch avg over {n[k]} rows)")
PY
cat $OUT/t.txt | grep -v amdgpu.ids
