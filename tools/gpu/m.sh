set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 100 python tools/gpu/micro.py metrics && RSX_LIB=$PWD/recommendar-systems_amd/rsx/lib/variants/mold/librsx.so timeout -k 10 100 python tools/gpu/micro.py metrics
