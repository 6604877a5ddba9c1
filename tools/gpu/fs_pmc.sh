set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/fpmc
A="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_MFMA"
B="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_SCA"
for m in 0 1; do
  i=0
  for set in "$A" "$B"; do
    i=$((i+1))
    RSX_FS_NUSERS=32768 RSX_FS_MODE=$m timeout -k 10 200 rocprofv3 --pmc $set --kernel-include-regex fs_tiles --output-format csv -d gpurun_out/fpmc/m${m}_$i -o p -- python tools/gpu/micro.py fullsort > /dev/null 2>&1 || exit 1
  done
done
echo done
