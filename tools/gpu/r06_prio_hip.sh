# round 6: the priority-stream fault without RCCL or torch
# (tools/gpu/exp/prio_destroy.hip); stops at the first failing variant
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/r06priohip}
mkdir -p "$OUT"
run() {
  timeout -k 10 60 tools/gpu/exp/prio_destroy "$@" >> "$OUT/prio_destroy.txt" 2>&1
  rc=$?
  echo "variant prio=$1 destroy=$2 eager=$3 rc=$rc" | tee -a "$OUT/prio_destroy.txt"
  return $rc
}
run 0 1 1 && run 1 0 1 && run 1 1 0 && run 1 1 1
echo done
