# Build librsx variants differing only in fullsort.hip's compile-time knobs:
#   tools/build_variant.sh NAME "-DRSX_FS_ABUF=2 ..."  -> recommendar-systems_amd/rsx/lib/var/NAME.so
# (select one on the GPU box with RSX_LIB=recommendar-systems_amd/rsx/lib/var/NAME.so)
set -e
cd "$(dirname "$0")/.."
P=recommendar-systems_amd
mkdir -p $P/rsx/lib/var
python -c "import sys; sys.path.insert(0, '$P'); from rsx import build; build.build(verbose=False)"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Iinclude -I$P/csrc $2 -c $P/csrc/fullsort.hip -o /tmp/fs_$1.o
objs=$(ls $P/rsx/lib/obj/*.o | grep -v fullsort.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $P/rsx/lib/var/$1.so $objs /tmp/fs_$1.o -ldl
echo built $P/rsx/lib/var/$1.so
