# round 6: selected GPU tests (TESTS="file[::k] ..."; K = -k expression), one pytest process
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/r06t}
mkdir -p "$OUT"
timeout -k 10 ${TO:-900} python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread ${K:+-k "$K"} \
  > "$OUT/pytest.log" 2>&1 || { tail -60 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
