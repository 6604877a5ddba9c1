set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_smore.py -q -x -p no:cacheprovider 2>&1 | tail -30
