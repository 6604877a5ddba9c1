"""Build a variant of librsx.so with extra flags (-D..., -mllvm ...) on every source into
rsx/lib/variants/<name>/
(for side-by-side timing on the GPU box via RSX_LIB=...).
usage: python tools/build_variant.py NAME -DFOO=1 [-DBAR=2 ...]"""
import os
import subprocess
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "recommendar-systems_amd"))
from rsx import build as B  # noqa: E402

name, defs = sys.argv[1], sys.argv[2:]
out = os.path.join(B.LIBDIR, "variants", name)
os.makedirs(out, exist_ok=True)
objs = []
for src in B.SOURCES:
    obj = os.path.join(out, os.path.splitext(src)[0] + ".o")
    if src.endswith(".cpp"):  # host code, as rsx.build compiles it
        cmd = [B._hipcc(), "-x", "c++", "-O3", "-fPIC", "-std=c++17", "-pthread", f"-I{B.INCLUDE}", f"-I{B.CSRC}",
               *defs, "-c", os.path.join(B.CSRC, src), "-o", obj]
    else:
        cmd = [B._hipcc(), *B._flags(src), *defs, "-c", os.path.join(B.CSRC, src), "-o", obj]
    subprocess.run(cmd, check=True)
    objs.append(obj)
subprocess.run([B._hipcc(), f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-pthread", "-o",
                os.path.join(out, "librsx.so"), *objs, "-ldl"], check=True)
print(os.path.join(out, "librsx.so"))
