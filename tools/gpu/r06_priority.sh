# round 6: the priority-stream capture fault; every variant in its own
# process (a host segfault ends only that process)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/r06prio}
mkdir -p "$OUT"
ALL=a0d0g1,a0d0g0,a0d1g1,a0d1g0,a1d0g1,a1d0g0,a1d1g1,a1d1g0
run() {  # name prio combos
  timeout -k 10 150 python -X faulthandler tools/gpu/diag_priority2.py $2 $3 > "$OUT/$1.txt" 2>&1
  echo "$1 rc=$? $(grep -c ' ok ' "$OUT/$1.txt") steps ok; last: $(grep -v '^ *File\|^  ' "$OUT/$1.txt" | tail -1)"
}
run prio1_all 1 $ALL
run prio0_all 0 $ALL
run prio1_graphs 1 a0d0g1,a0d1g1,a1d0g1,a1d1g1
for c in a0d0g1 a0d1g1 a1d0g1 a1d1g1; do run prio1_$c 1 $c; done
run prio1_a0d0g1x2 1 a0d0g1,a0d0g1
echo done
