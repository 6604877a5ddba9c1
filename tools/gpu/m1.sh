set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python tools/gpu/micro.py floor && \
for b in 1024 4096; do RSX_SPMM_MAXB=$b timeout -k 10 200 python tools/gpu/micro.py floor || exit 1; echo "maxb $b"; done
