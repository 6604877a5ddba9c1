# round 6: the round-5 segfault's own test pattern (_sim_worker); each
# variant in its own process, stop at the first fault (a segfault is a host-side crash in
# hipGraphLaunch, not a GPU fault, but nothing more runs after one)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/r06prio3}
mkdir -p "$OUT"
run() {  # name prio seq [close]
  timeout -k 10 150 python -X faulthandler tools/gpu/diag_priority3.py $2 $3 $4 > "$OUT/$1.txt" 2>&1
  rc=$?
  echo "$1 rc=$rc $(grep -c ' ok ' "$OUT/$1.txt") steps ok; last: $(grep '^\[' "$OUT/$1.txt" | tail -1)"
  return $rc
}
if [ -n "$STAGE4" ]; then
  export RSX_DIAG_SEGV_BT=1
  [ -z "$SKIP_STREAM" ] && RSX_COMM_DIAG_KEEP=1 run prio1_keep_stream 1 real,sim;
  [ -z "$SKIP_EVENTS" ] && RSX_COMM_DIAG_KEEP=4 run prio1_keep_events 1 real,sim;
  RSX_COMM_DIAG_KEEP=2 run prio1_keep_rccl 1 real,sim
elif [ -n "$STAGE3" ]; then
  export RSX_DIAG_SEGV_BT=1
  run prio1_real_sim_leak 1 real,sim leak &&
  RSX_COMM_PRIORITY=0 run noprio_real_sim 0 real,sim &&
  run prio1_real_sim_bt 1 real,sim
elif [ -n "$STAGE2" ]; then
  run prio1_real_sim_drain 1 real,sim drain &&
  run prio1_real_sim_leak 1 real,sim leak &&
  RSX_COMM_PRIORITY=0 run noprio_real_sim 0 real,sim &&
  run prio1_real_real 1 real,real
else
  run prio0_real_sim 0 real,sim &&
  run prio1_sim 1 sim &&
  run prio1_real 1 real &&
  run prio1_real_sim 1 real,sim
fi
echo done
