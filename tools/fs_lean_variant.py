"""Rebuild the reverted round-2 'leaner masked-tile branch' of fs_screen's pass 2 as a
side library (rsx/lib/variants/fs_lean/librsx.so) to pin down which invariant it broke
(csrc/fullsort.hip, "Invariants", (iv)): the variant never queues a masked item.

usage: python tools/fs_lean_variant.py   -> prints the library path; then on the GPU box
  RSX_LIB=<path> python -m pytest tests/test_gpu_realshape.py -m gpu -k screen_exact_vs_cpu
fails on the masked-heavy users (every other row stays exact)."""
import os
import shutil
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "recommendar-systems_amd"))
from rsx import build as B  # noqa: E402

PASS2_MASKED = "                push((v > tv) & (io < remh), (ebase + ((unsigned)io << 6)) | (msk ? 32u : 0u));"
LEAN = "                push(!msk & (acc[r] > tv) & (io < remh), ebase + ((unsigned)io << 6));"

tmp = tempfile.mkdtemp(prefix="fs_lean_")
for f in os.listdir(B.CSRC):
    shutil.copy(os.path.join(B.CSRC, f), tmp)
src = open(os.path.join(tmp, "fullsort.hip")).read()
if PASS2_MASKED not in src:
    raise SystemExit("pass-2 masked-tile push not found: update PASS2_MASKED")
open(os.path.join(tmp, "fullsort.hip"), "w").write(src.replace(PASS2_MASKED, LEAN))
out = os.path.join(B.LIBDIR, "variants", "fs_lean")
os.makedirs(out, exist_ok=True)
objs = []
for s in B.SOURCES:
    obj = os.path.join(out, s.replace(".hip", ".o"))
    subprocess.run([B._hipcc(), *B._flags(), f"-I{tmp}", "-c", os.path.join(tmp, s), "-o", obj], check=True)
    objs.append(obj)
subprocess.run([B._hipcc(), f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", os.path.join(out, "librsx.so"),
                "-ldl", *objs], check=True)
shutil.rmtree(tmp)
print(os.path.join(out, "librsx.so"))
