"""librsx.so loads here (no GPU) and exports every entry point include/rsx.h declares;
the host-side schedule builder is exercised directly."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from rsx import _lib as L

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(REPO, "include", "rsx.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rsx_[a-z0-9_]+)\s*\(", src)))


def test_exports_every_declared_symbol():
    lib = L.lib()
    names = _declared()
    assert len(names) >= 13
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(L.EXPORTED) <= set(names)
    assert lib.rsx_version().decode().startswith("rsx ")


def test_struct_layouts_match_header(tmp_path):
    """The ctypes mirrors have the sizes gcc gives the C structs of include/rsx.h (a
    field added on one side only shifts every later field)."""
    import shutil
    import subprocess

    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    inc = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "include")
    src = tmp_path / "sz.c"
    src.write_text('#include "rsx.h"\n#include <stdio.h>\nint main(void){printf("%zu %zu %zu %zu %zu %zu %zu %zu",'
                   ' sizeof(rsx_csr), sizeof(rsx_adam), sizeof(rsx_epilogue), sizeof(rsx_lgcn_step),'
                   ' sizeof(rsx_sharded_lgcn_step), sizeof(rsx_sampler_args), sizeof(rsx_layergcn_step_args),'
                   ' sizeof(rsx_dp_lgcn_step));'
                   ' return 0;}\n')
    exe = tmp_path / "sz"
    subprocess.run([cc, "-I", inc, str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert got == [C.sizeof(L.Csr), C.sizeof(L.Adam), C.sizeof(L.Epilogue), C.sizeof(L.LgcnStep),
                   C.sizeof(L.ShardedStep), C.sizeof(L.SamplerArgs), C.sizeof(L.LayerGcnStep), C.sizeof(L.DpStep)]


def test_comm_unique_id_size():
    # the RCCL unique id the sharded step's handshake broadcasts (ncclUniqueId = 128 bytes)
    assert L.lib().rsx_comm_unique_id_bytes() == 128


def test_schedule_host_splits_hub_rows():
    lib = L.lib()
    deg = np.array([0, 3, 32, 33, 100, 0, 1])
    rowptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    nw, nl, ns = C.c_int64(), C.c_int64(), C.c_int64()
    rc = lib.rsx_csr_schedule_host(rowptr.ctypes.data_as(C.c_void_p), deg.size, 32, None, None,
                                   C.byref(nw), C.byref(nl), C.byref(ns))
    assert rc == 0
    assert (nw.value, nl.value, ns.value) == (4 + 2 + 4 + 1, 2, 6)
    work = np.zeros((nw.value, 4), np.int32)
    lr = np.zeros((nl.value, 4), np.int32)
    lib.rsx_csr_schedule_host(rowptr.ctypes.data_as(C.c_void_p), deg.size, 32, work.ctypes.data_as(C.c_void_p),
                              lr.ctypes.data_as(C.c_void_p), C.byref(nw), C.byref(nl), C.byref(ns))
    # every nonzero covered exactly once, chunks <= 32, slots contiguous per long row;
    # the long rows' chunks come first (x = long-row index), whole rows after them
    cover = np.zeros(rowptr[-1], np.int32)
    assert lr.tolist() == [[3, 0, 2, 0], [4, 2, 4, 0]]
    n_chunks = int(lr[:, 2].sum())
    for i, (x, slot, b, e) in enumerate(work):
        r = lr[x, 0] if i < n_chunks else x
        assert (slot >= 0) == (i < n_chunks)
        if slot >= 0:
            assert lr[x, 1] <= slot < lr[x, 1] + lr[x, 2]
        assert 0 <= e - b <= 32 and rowptr[r] <= b <= e <= rowptr[r + 1]
        cover[b:e] += 1
    assert np.all(cover == 1)
    # nnz >= 2^31 is refused (32-bit work offsets)
    big = np.array([0, 1 << 31], dtype=np.int64)
    assert lib.rsx_csr_schedule_host(big.ctypes.data_as(C.c_void_p), 1, 32, None, None, C.byref(nw),
                                     C.byref(nl), C.byref(ns)) == 1001


@pytest.mark.parametrize("nb,ni,d,chunks,per", [
    (35598, 18357, 64, 2, 9184),      # C2: two chunks, the balanced split (2,226 waves > 2,048 slots)
    (19445, 7050, 64, 3, 2368),       # baby: three chunks fill 89 % of the slots in one round
    (39387, 23033, 128, 2, 11520),    # C5
    (4096, 18357, 64, 16, 1152),      # few users: 16 chunks (lists cut to top k)
    (16384, 400000, 256, 2, 200000),  # C4-like d = 256 (one wave per SIMD)
    (40, 500, 64, 16, 32),            # tiny: at most 16 chunks
])
def test_fullsort_plan_host(nb, ni, d, chunks, per):
    """The screened full-sort's item-chunk plan (csrc/fullsort.hip screen_plan, 256 CUs
    assumed without a GPU), as rsx_fullsort_plan reports it."""
    nc, pi = C.c_int32(), C.c_int64()
    L.check(L.lib().rsx_fullsort_plan(nb, ni, d, C.byref(nc), C.byref(pi)), "rsx_fullsort_plan")
    assert (nc.value, pi.value) == (chunks, per)


def test_row_slice_schedules_cover_the_parent_rows():
    """DeviceCSR.row_slice (the sharded step's head pieces, rsx_sharded_lgcn_step.n_head):
    each piece's schedule is the host schedule of its rows, row ids local to the piece,
    nonzero offsets into the parent's col / val; the pieces' work items together cover
    every nonzero of the parent once, in the same chunks."""
    from rsx import ops
    from rsx.dist import head_pieces_knob

    rng = np.random.default_rng(5)
    deg = np.concatenate([rng.integers(0, 12, 300), [0, 33, 64, 65, 200, 1000]])
    rng.shuffle(deg)
    rowptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    nnz = int(rowptr[-1])
    col = rng.integers(0, 500, nnz).astype(np.int32)
    val = rng.random(nnz).astype(np.float32)
    parent = ops.DeviceCSR(rowptr, col, val, 500, "cpu", chunk=32)
    cuts = [0, 77, 150, 151, rowptr.size - 1]
    seen = np.zeros(nnz, np.int32)
    for a, b in zip(cuts[:-1], cuts[1:]):
        piece = ops.DeviceCSR.row_slice(parent, a, b)
        assert piece.n_rows == b - a and piece.col is parent.col and piece.val is parent.val
        work = piece.work.numpy()[: piece.n_work]
        lr = piece.long_rows.numpy()[: piece.n_long]
        n_chunks = int(lr[:, 2].sum()) if piece.n_long else 0
        for i, (x, slot, s, e) in enumerate(work):
            r = (lr[x, 0] if i < n_chunks else x) + a  # the parent's row
            assert rowptr[r] <= s <= e <= rowptr[r + 1] and e - s <= 32
            seen[s:e] += 1
    assert (seen == 1).all()
    assert head_pieces_knob(4) == 4
    import os

    os.environ["RSX_SHARDED_HEAD"] = "x"
    try:
        with pytest.raises(ValueError):
            head_pieces_knob(4)
    finally:
        del os.environ["RSX_SHARDED_HEAD"]
