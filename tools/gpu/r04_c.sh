# round 4, batch C: SMORE tests + C5 / C3 lines (ego table without the cat, rsx_tag_rows),
# the C4 W = 8 latency-injected step trace, the data-parallel C2 leg at one rank
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu/r04_smore.sh && W=8 bash tools/gpu/c4_simtrace.sh && bash tools/gpu/r04_dpm.sh
