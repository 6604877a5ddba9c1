"""Build librsx.so (the gfx950 HIP kernels + C ABI) in-tree with hipcc.

`python -m rsx.build` or `rsx.build.build()`; `__graft_entry__.build()` calls this.
The library lands in `rsx/lib/librsx.so` so it travels with the repository
snapshot to the GPU box (no JIT cache, no site-packages install).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)  # recommendar-systems_amd/
REPO = os.path.dirname(ROOT)
CSRC = os.path.join(ROOT, "csrc")
INCLUDE = os.path.join(REPO, "include")
LIBDIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIBDIR, "librsx.so")
SOURCES = ["spmm.hip", "bpr.hip", "fullsort.hip", "step.hip", "smore.hip", "metrics.hip", "linear.hip", "dist.hip",
           "dp.hip", "smore_fuse.hip", "knn.hip", "graph.hip", "rowx.hip",
           "cpu_ops.cpp"]  # host-only C++ (the torch.ops.rsx CPU kernels), compiled as plain C++
ARCH = os.environ.get("RSX_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: librsx.so needs ROCm's hipcc (gfx950)")


# Per-source code-generation flags.  -amdgpu-mfma-vgpr-form: MFMA accumulators in the
# architectural VGPRs.  Without it the register allocator keeps a loop-carried
# accumulator in VGPRs and copies it into AGPRs and back around every MFMA block
# (wgrad_partial<2,4,DX>: 64 v_accvgpr moves per two-chunk step, 156 VGPRs + AGPRs);
# with it the kernel has no AGPR traffic and 118 VGPRs.  Same instructions otherwise,
# so the results are bit-identical.
SOURCE_FLAGS = {
    "linear.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"],
}


def _flags(src: str | None = None):
    return [f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", f"-I{INCLUDE}", f"-I{CSRC}",
            "-Wno-unused-result", *SOURCE_FLAGS.get(src, [])]


def _needs_build() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + [os.path.join(INCLUDE, "rsx.h"), __file__]
    return any(os.path.getmtime(p) > t for p in deps if os.path.isfile(p))


def build(force: bool = False, verbose: bool = True) -> str:
    """Compile every HIP source for gfx950 and link librsx.so; returns its path."""
    if not force and not _needs_build():
        return LIB
    hipcc = _hipcc()
    objdir = os.path.join(PKG, "lib", "obj")
    os.makedirs(objdir, exist_ok=True)
    srcs = [s for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]

    def compile_one(src):
        obj = os.path.join(objdir, os.path.splitext(src)[0] + ".o")
        if src.endswith(".cpp"):  # host code: no device pass
            # x86-64-v3 (AVX2 + FMA): every host these runs use (EPYC GPU boxes, this Xeon) has it
            cmd = [hipcc, "-x", "c++", "-O3", "-march=x86-64-v3", "-fPIC", "-std=c++17", "-pthread", f"-I{INCLUDE}",
                   f"-I{CSRC}", "-c", os.path.join(CSRC, src), "-o", obj]
        else:
            cmd = [hipcc, *_flags(src), "-c", os.path.join(CSRC, src), "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
        return obj

    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(compile_one, srcs))
    tmp = LIB + ".tmp"
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-pthread", "-o", tmp, *objs, "-ldl"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    os.replace(tmp, LIB)
    if verbose:
        print(f"[rsx.build] built {LIB}", file=sys.stderr)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
